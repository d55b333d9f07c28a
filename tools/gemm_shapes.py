"""Prefill GEMM sweep: ops.linear over (M, N, K) shapes, HIP-event time per
launch and TFLOP/s / output GB/s."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops

BF = torch.bfloat16


def timeit(fn, reps=10):
  """Device time per launch: `reps` launches captured in one hipGraph (no
  host launch overhead in the measurement)."""
  fn(); torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay(); torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  g.replay()
  e.record(); torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  dev = torch.device("cuda")
  shapes = [tuple(int(v) for v in s.split("x")) for s in
            os.environ.get("SHAPES", "10208x5120x256,10208x5120x64,10208x256x256,"
                           "2048x5120x256,10208x5120x2560,10208x2560x2560,"
                           "10208x2560x7680,8352x1024x1024,8352x3072x1024,"
                           "8192x4352x1152").split(",")]
  tag = "big"
  for M, N, K in shapes:
    if os.environ.get("UNIFORM") == "1":   # uniform [-1, 1) operands
      a = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
      w = (torch.rand(N, K, device=dev) * 2 - 1).to(BF)
    else:
      a = torch.randn(M, K, device=dev).to(BF)
      w = (torch.randn(N, K, device=dev) / K ** .5).to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    us = timeit(lambda: ops.linear(a, w, out=out))
    print(f"{tag:6s} M={M:6d} N={N:6d} K={K:5d} {us:8.1f} us "
          f"{2*M*N*K/us/1e6:7.1f} TF/s  out {M*N*2/us/1e3:6.0f} GB/s", flush=True)
    if os.environ.get("VS_TORCH") == "1":   # hipBLASLt through torch.mm
      wt = w.t()
      us = timeit(lambda: torch.mm(a, wt, out=out))
      print(f"torch  M={M:6d} N={N:6d} K={K:5d} {us:8.1f} us "
            f"{2*M*N*K/us/1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
  main()
