"""Bitwise A/B of the gated-GELU prefill GEMM between two builds of the
library (an epilogue rewrite must not move a single output bit): loads both
.so files by ctypes (separate handles), runs cadence_gemm_gated_gelu on the
same device buffers under each engine plan (mask 3: the 4-wave engine where
planned, 2: the 8-wave engine), and times each (HIP events, 10 launches).
usage: python tools/epi_bitwise.py OLD.so NEW.so"""
import ctypes
import sys

import torch

P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float


def load(path):
  lib = ctypes.CDLL(path)
  f = lib.cadence_gemm_gated_gelu
  f.argtypes = [P, I64, P, I64, P, P, P, I64, I64, I64, I64, P, I64, I32, F32, P]
  f.restype = I32
  lib.cadence_gemm_set_engine.argtypes = [I32]
  lib.cadence_gemm_set_engine.restype = I32
  lib.cadence_gemm_workspace_bytes.argtypes = [I64, I64, I64, I64]
  lib.cadence_gemm_workspace_bytes.restype = I64
  return lib


def run(lib, x, w, bg, bu, out, ws, M, F, K):
  st = torch.cuda.current_stream().cuda_stream
  rc = lib.cadence_gemm_gated_gelu(x.data_ptr(), K, w.data_ptr(), K, bg.data_ptr(),
                                   bu.data_ptr(), out.data_ptr(), F, M, F, K,
                                   ws.data_ptr(), ws.numel(), 0, 0.0, st)
  assert rc == 0, rc


def main():
  old, new = load(sys.argv[1]), load(sys.argv[2])
  dev = torch.device("cuda", 0)
  g = torch.Generator(device=dev).manual_seed(0)
  for M, F, K in ((10208, 7680, 2560), (20448, 7680, 2560), (8352, 2048, 1024),
                  (1000, 1024, 512)):
    x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(2 * F, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    bg = (torch.rand(F, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    bu = (torch.rand(F, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    nws = max(old.cadence_gemm_workspace_bytes(M, 2 * F, K, 1), 16)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    for eng in (3, 2):
      outs, times = [None, None], [1e30, 1e30]
      for rnd in range(4):            # alternate the builds, keep each one's best
        for li, lib in enumerate((old, new)):
          lib.cadence_gemm_set_engine(eng)
          out = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
          run(lib, x, w, bg, bu, out, ws, M, F, K)
          torch.cuda.synchronize()
          s, e = torch.cuda.Event(True), torch.cuda.Event(True)
          s.record()
          for _ in range(10):
            run(lib, x, w, bg, bu, out, ws, M, F, K)
          e.record()
          torch.cuda.synchronize()
          outs[li] = out
          times[li] = min(times[li], s.elapsed_time(e) / 10 * 1e3)
          lib.cadence_gemm_set_engine(7)
      eq = torch.equal(outs[0], outs[1])
      print(f"gated {M}x{2 * F}x{K} engine {eng}: bitwise equal {eq}  "
            f"old {times[0]:8.1f} us  new {times[1]:8.1f} us  ({times[0] / times[1]:.3f}x)",
            flush=True)


if __name__ == "__main__":
  main()
