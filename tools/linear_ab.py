"""Bitwise A/B of cadence_gemm_linear between two builds of the library (an
epilogue rewrite must not move a single output bit): loads both .so files by
ctypes, runs the prefill shapes of the bench (Griffin y|x and residual
projections, DINO / SigLIP q|k|v and MLP fc1 with GELU) on the same device
buffers, and times each build (HIP events, best of 4 alternated rounds of 10
launches).
usage: python tools/linear_ab.py OLD.so NEW.so"""
import ctypes
import sys

import torch

P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int


def load(path):
  lib = ctypes.CDLL(path)
  f = lib.cadence_gemm_linear
  f.argtypes = [P, I64, P, I64, P, P, I64, P, I64, I64, I64, I64, I32, I64, I64, I64,
                P, I64, P]
  f.restype = I32
  return lib


def run(lib, x, w, b, r, out, M, N, K, act):
  st = torch.cuda.current_stream().cuda_stream
  rc = lib.cadence_gemm_linear(x.data_ptr(), K, w.data_ptr(), K, b.data_ptr(),
                               r.data_ptr() if r is not None else None, N,
                               out.data_ptr(), N, M, N, K, act, M, 0, 0, None, 0, st)
  assert rc == 0, rc


def main():
  libs = load(sys.argv[1]), load(sys.argv[2])
  dev = torch.device("cuda", 0)
  g = torch.Generator(device=dev).manual_seed(0)
  BF = torch.bfloat16
  cases = (("griffin y|x", 10208, 5120, 2560, 0, False),
           ("griffin out + resid", 10208, 2560, 2560, 0, True),
           ("griffin down + resid", 10208, 2560, 7680, 0, True),
           ("dino qkv", 8352, 3072, 1024, 0, False),
           ("dino fc1 gelu", 8352, 4096, 1024, 1, False),
           ("siglip fc1 gelu-tanh", 8192, 4352, 1152, 3, False),
           ("small", 1000, 1024, 512, 0, False))
  for name, M, N, K, act, res in cases:
    x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(BF)
    w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).to(BF)
    b = (torch.rand(N, device=dev, generator=g) - 0.5).to(BF)
    r = (torch.rand(M, N, device=dev, generator=g) * 4 - 2).to(BF) if res else None
    outs, times = [None, None], [1e30, 1e30]
    for _ in range(4):
      for li, lib in enumerate(libs):
        out = torch.empty(M, N, dtype=BF, device=dev)
        run(lib, x, w, b, r, out, M, N, K, act)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(10):
          run(lib, x, w, b, r, out, M, N, K, act)
        e.record()
        torch.cuda.synchronize()
        outs[li] = out
        times[li] = min(times[li], s.elapsed_time(e) / 10 * 1e3)
    eq = torch.equal(outs[0], outs[1])
    print(f"{name:22s} {M}x{N}x{K} act {act}: bitwise equal {eq}  old {times[0]:8.1f} us  "
          f"new {times[1]:8.1f} us  ({times[0] / times[1]:.3f}x)", flush=True)


if __name__ == "__main__":
  main()
