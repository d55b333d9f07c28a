"""RG-LRU prefill gates microbenchmark (bench shape, M = 32 x 319 rows,
E = 2560, 10 blocks of 256): rglru_gates_stream_kernel (engine 1) against
the block engine it replaced (engine 0), HIP events around 20 launches;
HBM bytes = x in + a, normalised x out (+ the 2.6 MB of packed weights)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import _lib, ops

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
  lib = _lib.load()
  for M in (32 * 319, 319, 8 * 2048):
    E, H, bw = 2560, 10, 256
    yx = torch.randn(M, 2 * E, device=dev).to(BF)
    x = yx[:, E:]
    wg = (torch.randn(H, 2 * bw, bw, device=dev) / 16).to(BF)
    bx = torch.zeros(E, dtype=BF, device=dev)
    sp = torch.rand(E, device=dev).to(BF)
    pos = torch.randint(0, 50, (M,), dtype=torch.int32, device=dev)
    nbytes = 3 * M * E * 2 + wg.numel() * 2
    for eng in (3, 0):
      prev = lib.cadence_gemm_set_engine(eng)
      us = timeit(lambda: ops.ops.rglru_gates(x, wg, bx, bx, sp, pos))
      lib.cadence_gemm_set_engine(prev)
      print(f"M={M:6d} engine {eng}: {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s "
            f"({nbytes / us / 1e3 / 8000:.3f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
  main()
