"""A/B of the ViT attention kernels (cadence_gemm_set_engine bit 3: the
streaming vit_flash_attn_kernel for every size vs the round-3 LDS-resident /
streaming kernels) at the tower shapes, bs 32: device time per launch
(graph replays, rounds interleaved), MFMA fraction of 2.5 PF, rel-L2 of each
against an fp32 softmax(QK^T / sqrt(hd)) V.
usage: python tools/vit_flash_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import _lib, ops  # noqa: E402


def timeit(fn, reps=20):
  fn()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  g.replay()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
  dev = torch.device("cuda")
  lib = _lib.load()
  b = int(os.environ.get("B", "32"))
  base = lib.cadence_gemm_set_engine(-1)
  # the round-3 kernels and the shipped plan (bit 3: the flash kernel)
  ENGINES = (base & ~8, base | 8)
  shapes = (("dino224", 261, 16, 64), ("sig224", 256, 16, 72),
            ("dino336", 581, 16, 64), ("sig336", 576, 16, 72),
            ("dino384", 734, 16, 64), ("sig384", 729, 16, 72))
  cases = []
  for name, n, h, hd in shapes:
    g = torch.Generator(device=dev).manual_seed(5)
    qkv = (torch.randn(b * n, 3 * h * hd, device=dev, generator=g) * 1.5).to(torch.bfloat16)
    t = qkv.float().view(b, n, 3, h, hd).permute(2, 0, 3, 1, 4)
    att = torch.softmax((t[0] * hd ** -0.5) @ t[1].transpose(-1, -2), -1)
    want = (att @ t[2]).transpose(1, 2).reshape(b * n, h * hd)
    outs = {}
    for eng in ENGINES:
      lib.cadence_gemm_set_engine(eng)
      outs[eng] = ops.ops.vit_attention(qkv, b, n, h, hd)
      torch.cuda.synchronize()
    errs = [((outs[e].float() - want).norm() / want.norm()).item() for e in ENGINES]
    print(f"{name:8s} N={n} hd={hd}: rel_l2 " + " ".join(f"{x:.3e}" for x in errs), flush=True)
    cases.append((name, n, h, hd, qkv))
  times = {}
  for r in range(rounds):
    for name, n, h, hd, qkv in cases:
      for eng in ENGINES:
        lib.cadence_gemm_set_engine(eng)
        times.setdefault((name, eng), []).append(
            timeit(lambda: ops.ops.vit_attention(qkv, b, n, h, hd)))
  lib.cadence_gemm_set_engine(base)
  for name, n, h, hd, _ in cases:
    flops = 4.0 * b * h * n * n * hd
    med = [sorted(times[(name, e)])[rounds // 2] for e in ENGINES]
    print(f"{name:8s} " + "  ".join(f"{lbl} {t:7.2f} us ({flops / t / 1e6 / 2500:.3f})"
                                    for lbl, t in zip(("round-3", "plan"), med)),
          flush=True)


if __name__ == "__main__":
  main()
