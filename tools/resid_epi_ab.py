"""A/B of the prefill linear GEMM with a residual (the Griffin output and
down projections, cadence_gemm_linear act 0 + resid) between the plain
staged epilogue (engine mask 3) and EpiLinearA<4>, which loads the residual
rows before staging (mask 7): outputs must be bitwise equal; each plan's best
of 4 alternated rounds of 10 launches (HIP events).
usage: python tools/resid_epi_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402

from cadence import _lib, ops  # noqa: E402


def main():
  lib = _lib.load()
  dev = torch.device("cuda", 0)
  g = torch.Generator(device=dev).manual_seed(0)
  BF = torch.bfloat16
  for M, N, K in ((10208, 2560, 2560), (10208, 2560, 7680), (20448, 2560, 7680),
                  (65504, 2560, 2560), (1000, 1024, 512)):
    x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(BF)
    w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).to(BF)
    b = (torch.rand(N, device=dev, generator=g) - 0.5).to(BF)
    r = (torch.rand(M, N, device=dev, generator=g) * 4 - 2).to(BF)
    outs, times = [None, None], [1e30, 1e30]
    for _ in range(4):
      for li, eng in enumerate((3, 7)):
        prev = lib.cadence_gemm_set_engine(eng)
        out = ops.linear(x, w, b, resid=r)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(10):
          ops.linear(x, w, b, resid=r, out=out)
        e.record()
        torch.cuda.synchronize()
        lib.cadence_gemm_set_engine(prev)
        outs[li] = out
        times[li] = min(times[li], s.elapsed_time(e) / 10 * 1e3)
    eq = torch.equal(outs[0], outs[1])
    tf = 2 * M * N * K / times[1] / 1e6
    print(f"linear+resid {M}x{N}x{K}: bitwise equal {eq}  plain {times[0]:8.1f} us  "
          f"prefetch {times[1]:8.1f} us  ({times[0] / times[1]:.3f}x, {tf:.0f} TFLOP/s)",
          flush=True)


if __name__ == "__main__":
  main()
