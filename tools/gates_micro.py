"""RG-LRU gate GEMM microbenchmark (prefill shape, M = 32 x 319 rows):
the fused gate chain vs plain GEMMs of the same operand shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops

BF = torch.bfloat16


def timeit(fn, reps=20):
  fn(); torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps):
    fn()
  e.record(); torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  dev = torch.device("cuda")
  M = int(os.environ.get("M", str(32 * 319)))
  E, H, bw = 2560, 10, 256
  x = torch.randn(M, E, device=dev).to(BF)
  wg = (torch.randn(H, 2 * bw, bw, device=dev) / 16).to(BF)
  bx = torch.zeros(E, dtype=BF, device=dev)
  pos = torch.ones(M, dtype=torch.int32, device=dev)
  w1 = wg[0].contiguous()
  wbig = torch.randn(5120, 256, device=dev).to(BF)
  xs = x[:, :256]
  cases = [
      ("rglru_gates (10 groups)", lambda: ops.ops.rglru_gates(x, wg, bx, bx, bx, pos)),
      ("linear N=512 K=256 x10", lambda: [ops.linear(xs, w1) for _ in range(10)]),
      ("linear N=5120 K=256", lambda: ops.linear(xs, wbig)),
      ("linear N=5120 K=2560", lambda: ops.linear(x, wx)),
  ]
  global wx
  wx = torch.randn(5120, 2560, device=dev).to(BF)
  for name, fn in cases:
    print(f"{name:28s} {timeit(fn):9.1f} us", flush=True)


if __name__ == "__main__":
  main()
