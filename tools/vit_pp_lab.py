"""The phase-locked 8-wave ViT attention lab (tools/vit_pp_kernel.hip)
against the 32x32 persistent kernel it restructures (vit_fa32_kernel, lab
-1): outputs compared (bitwise and rel-L2 to an fp32 reference of the same
pre-scaled q), then device time per launch over graph replays for the
product variant (lab 0) and its measurement variants (2 no exp, 8 no P.V
MFMAs, 16 no QK^T MFMAs, 24 no MFMA, 32 no s_setprio on the MFMA phase).
usage: python tools/vit_pp_lab.py [shape ...]   (hd 64 shapes: dino224/336/384)"""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

LIB = os.path.join(ROOT, "tools", "_build", "libpplab.so")
SHAPES = {"dino224": 261, "dino336": 581, "dino384": 734}


def timeit(fn, reps=20):
  fn()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  best = 1e9
  for _ in range(3):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    best = min(best, s.elapsed_time(e) / reps * 1e3)
  return best


def main():
  lib = ctypes.CDLL(LIB)
  lib.pp_lab.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int64] * 4 + \
      [ctypes.c_int, ctypes.c_void_p]
  dev = torch.device("cuda")
  b, h, hd = 32, 16, 64
  names = sys.argv[1:] or ["dino336", "dino224", "dino384"]
  for name in names:
    n = SHAPES[name]
    torch.manual_seed(0)
    qkv = (torch.randn(b * n, 3 * h * hd, device=dev) * 0.5).to(torch.bfloat16)
    outs = {}
    for lab in (-1, 0, 256, 768):
      o = torch.zeros(b * n, h * hd, device=dev, dtype=torch.bfloat16)
      rc = lib.pp_lab(qkv.data_ptr(), o.data_ptr(), b, n, h, hd, lab,
                      torch.cuda.current_stream().cuda_stream)
      torch.cuda.synchronize()
      assert rc == 0, (name, lab, rc)
      outs[lab] = o
    # fp32 reference: q already holds q * hd^-1/2 * log2(e)
    x = qkv.float().view(b, n, 3, h, hd)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    p = torch.softmax((q @ k.transpose(-1, -2)) * math.log(2.0), dim=-1)
    ref = (p @ v).transpose(1, 2).reshape(b * n, h * hd)
    rel = lambda o: float((o.float() - ref).norm() / ref.norm())
    for lab in (0, 256, 768):
      print(f"{name}: pp lab {lab} vs fa32 bitwise {torch.equal(outs[lab], outs[-1])}, max|d| "
            f"{(outs[lab].float() - outs[-1].float()).abs().max().item():.3g}; rel-L2 to fp32 "
            f"pp {rel(outs[lab]):.3e} fa32 {rel(outs[-1]):.3e}", flush=True)
    flops = 4.0 * b * h * n * n * hd
    out = torch.empty(b * n, h * hd, device=dev, dtype=torch.bfloat16)
    for lab in (-1, 0, 32, 256, 288, 768, 800, 770, 776, 784, 792):
      run = lambda lab=lab: lib.pp_lab(qkv.data_ptr(), out.data_ptr(), b, n, h, hd, lab,
                                       torch.cuda.current_stream().cuda_stream)
      us = timeit(run)
      print(f"{name:8s} {'fa32' if lab < 0 else 'pp lab=%d' % lab:12s}: {us:8.2f} us  "
            f"({flops / us / 1e6 / 2500:.3f} of 2.5 PF)", flush=True)


if __name__ == "__main__":
  main()
