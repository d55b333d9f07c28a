"""Conv1D prefill microbenchmark at the bench shape (B = 32, L = 319,
E = 2560, the packed [y | x] layout: ldx = 2E) and C2's (L = 2048), graph-
replayed; bytes = x in + y out (bf16).  usage: python tools/conv_micro.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import _lib


def timeit(fn, reps=20):
  st = torch.cuda.Stream()
  st.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(st):
    fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
      for _ in range(reps):
        fn()
  torch.cuda.current_stream().wait_stream(st)
  g.replay(); torch.cuda.synchronize()
  s, t = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record(); g.replay(); t.record(); torch.cuda.synchronize()
  return s.elapsed_time(t) / reps * 1e3


def main():
  dev = torch.device("cuda")
  lib = _lib.load()
  e = 2560
  for b, l in ((32, 319), (32, 2048)):
    m = b * l
    yx = torch.randn(m, 2 * e, device=dev).to(torch.bfloat16)
    w = torch.randn(4, e, device=dev).to(torch.bfloat16)
    bias = torch.randn(e, device=dev).to(torch.bfloat16)
    pos = torch.arange(l, dtype=torch.int32, device=dev)[None].repeat(b, 1)
    pos[:, 256:] -= 256          # a document start inside the rows (bench splice)
    out = torch.empty(m, e, device=dev, dtype=torch.bfloat16)
    cache = torch.empty(b, 3, e, device=dev, dtype=torch.bfloat16)
    fn = lambda: lib.cadence_conv1d(
        yx[:, e:].data_ptr(), 2 * e, w.data_ptr(), bias.data_ptr(), pos.data_ptr(),
        None, out.data_ptr(), e, cache.data_ptr(), b, l, e, 4, 1,
        torch.cuda.current_stream().cuda_stream)
    us = timeit(fn)
    print(f"conv1d B {b} L {l:5d} E {e}: {us:7.1f} us  {m * e * 4 / us / 1e3:7.0f} GB/s",
          flush=True)


if __name__ == "__main__":
  main()
