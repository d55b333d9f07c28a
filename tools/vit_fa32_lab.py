"""Where vit_fa32_kernel's time goes: the product kernel against variants
with parts removed (tools/vit_fa32_lab.hip LAB bits: 1 no per-tile DMA, 2 no
exp, 4 no max check, 8 no P.V MFMAs, 16 no QK^T MFMAs) and ring depths, at
the tower shapes, bs 32 (device time per launch over graph replays).
usage: python tools/vit_fa32_lab.py [shape ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

LIB = os.path.join(ROOT, "tools", "_build", "libfa32lab.so")


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
  lib.fa32_lab.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int64] * 4 + \
      [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
  dev = torch.device("cuda")
  b = 32
  shapes = {"dino224": (261, 16, 64), "sig224": (256, 16, 72), "dino336": (581, 16, 64),
            "sig336": (576, 16, 72), "dino384": (734, 16, 64), "sig384": (729, 16, 72)}
  args = sys.argv[1:]
  if args and args[0] == "--pmc":
    # a profiler target: the product variant (lab 0) of one shape, 20 plain launches
    n, h, hd = shapes[args[1]]
    qkv = (torch.randn(b * n, 3 * h * hd, device=dev) * 0.5).to(torch.bfloat16)
    out = torch.empty(b * n, h * hd, device=dev, dtype=torch.bfloat16)
    for _ in range(20):
      lib.fa32_lab(qkv.data_ptr(), out.data_ptr(), b, n, h, hd, int(args[2]) if len(args) > 2
                   else 0, 4, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return
  names = args or ["dino336", "sig336", "dino224"]
  labs = [0, 64, 96, 32, 1, 2, 4, 8, 16, 24, 31]
  for name in names:
    n, h, hd = shapes[name]
    qkv = (torch.randn(b * n, 3 * h * hd, device=dev) * 0.5).to(torch.bfloat16)
    out = torch.empty(b * n, h * hd, device=dev, dtype=torch.bfloat16)
    flops = 4.0 * b * h * n * n * hd
    for nb in (3, 4):
      for lab in labs:
        run = lambda: lib.fa32_lab(qkv.data_ptr(), out.data_ptr(), b, n, h, hd, lab, nb,
                                   torch.cuda.current_stream().cuda_stream)
        if run() != 0:
          print(name, "launch failed", lab, nb)
          continue
        us = timeit(run)
        print(f"{name:8s} nb={nb} lab={lab:2d}: {us:8.2f} us  ({flops / us / 1e6 / 2500:.3f})",
              flush=True)


if __name__ == "__main__":
  main()
