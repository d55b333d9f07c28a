"""Does a CU-masked stream (hipExtStreamCreateWithCUMask) restrict direct
launches and hipGraph replays, and how do the mask bits map to CUs?  Times a
prefill GEMM (10208 x 5120 x 2560) launched directly and replayed from a
graph on streams with 1/8 .. 8/8 of the mask bits set, in two bit patterns
(every 8th bit group: b % 8 < e; contiguous: b < 32 e).

usage: python tools/cumask_probe.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import _lib, ops  # noqa: E402


def masked_stream(hip, bits):
  words = [0] * 8
  for b in bits:
    words[b // 32] |= 1 << (b % 32)
  arr = (ctypes.c_uint32 * 8)(*words)
  s = ctypes.c_void_p()
  rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, arr)
  assert rc == 0, rc
  return torch.cuda.ExternalStream(s.value)


def main():
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  hip = ctypes.CDLL(_lib.hip_runtimes_loaded()[0])
  M, N, K = 10208, 5120, 2560
  a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
  w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
  out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
  run = lambda: ops.linear(a, w, out=out)
  run()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  cap = torch.cuda.Stream(device=dev)
  with torch.cuda.stream(cap):
    with torch.cuda.graph(g, stream=cap):
      for _ in range(5):
        run()
  torch.cuda.synchronize()

  def t_on(s, fn, reps=5):
    with torch.cuda.stream(s):
      fn()
      e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
      e0.record()
      for _ in range(reps):
        fn()
      e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3

  for pat in ("mod8", "contig"):
    for e in (8, 7, 4, 2, 1):
      bits = [b for b in range(256) if ((b % 8) < e if pat == "mod8" else b < 32 * e)]
      s = masked_stream(hip, bits)
      direct = t_on(s, run)
      graph = t_on(s, g.replay) / 5
      print(f"{pat:6s} {e}/8 bits: direct {direct:8.1f} us   graph replay {graph:8.1f} us",
            flush=True)


if __name__ == "__main__":
  main()
