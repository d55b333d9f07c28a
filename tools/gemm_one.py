"""One prefill GEMM shape launched REPS times back to back (for rocprofv3
--pmc / --kernel-trace runs of a single kernel): EPI=linear|gelu|gated, SHAPE=MxNxK.
Random operands (DVFS: zero-filled data runs at a higher clock)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops

BF = torch.bfloat16


def main():
  dev = torch.device("cuda")
  M, N, K = (int(v) for v in os.environ.get("SHAPE", "10208x15360x2560").split("x"))
  epi = os.environ.get("EPI", "gated")
  reps = int(os.environ.get("REPS", "20"))
  torch.manual_seed(0)
  a = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
  w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** .5).to(BF)
  if epi == "gated":
    bg = torch.zeros(N // 2, device=dev, dtype=BF)
    fn = lambda: ops.ops.gated_gelu(a, w, bg, bg)
  else:   # linear (no activation) or gelu (erf GELU epilogue, ViT fc1)
    out = torch.empty(M, N, device=dev, dtype=BF)
    act = 1 if epi == "gelu" else 0
    fn = lambda: ops.linear(a, w, act=act, out=out)
  fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps):
    fn()
  e.record()
  torch.cuda.synchronize()
  us = s.elapsed_time(e) / reps * 1e3
  flop = (4.0 * M * (N // 2) * K) if epi == "gated" else 2.0 * M * N * K
  print(f"{epi} M={M} N={N} K={K}: {us:.1f} us  {flop / us / 1e6:.1f} TF/s", flush=True)


if __name__ == "__main__":
  main()
