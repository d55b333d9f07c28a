"""Probe: does a HIP stream created with a CU mask (hipExtStreamCreateWithCUMask)
confine kernels -- eager launches and hipGraph replays -- to those CUs?
Times one prefill GEMM on the default stream and on streams masked to
1/2 and 1/4 of the CUs (mask bits spread over all XCDs)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops

BF = torch.bfloat16


def masked_stream(dev, keep):
  """torch ExternalStream over a HIP stream limited to CUs i with keep(i)."""
  hip = ctypes.CDLL("libamdhip64.so")
  n = torch.cuda.get_device_properties(dev).multi_processor_count
  words = (n + 31) // 32
  mask = (ctypes.c_uint32 * words)()
  for i in range(n):
    if keep(i):
      mask[i // 32] |= 1 << (i % 32)
  s = ctypes.c_void_p()
  rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
  assert rc == 0, f"hipExtStreamCreateWithCUMask rc {rc}"
  return torch.cuda.ExternalStream(s.value, device=dev)


def timeit(fn, stream, reps=10, graph=False):
  with torch.cuda.stream(stream):
    fn()
    torch.cuda.synchronize()
    if graph:   # captured on a plain side stream, replayed on `stream`
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g, stream=torch.cuda.Stream(device=stream.device)):
        for _ in range(reps):
          fn()
      run = g.replay
    else:
      def run():
        for _ in range(reps):
          fn()
    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record(stream)
    run()
    e.record(stream)
    torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  M, N, K = 10208, 5120, 2560
  a = (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
  w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** .5).to(BF)
  out = torch.empty(M, N, device=dev, dtype=BF)
  fn = lambda: ops.linear(a, w, out=out)
  base = torch.cuda.current_stream(dev)
  for name, st in (("default", base),
                   ("half (even CUs)", masked_stream(dev, lambda i: i % 2 == 0)),
                   ("quarter (i%4==0)", masked_stream(dev, lambda i: i % 4 == 0))):
    for graph in (False, True):
      us = timeit(fn, st, graph=graph)
      print(f"{name:18s} {'graph' if graph else 'eager'}  {us:8.1f} us", flush=True)


if __name__ == "__main__":
  main()
