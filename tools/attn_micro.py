"""Griffin prefill local attention microbenchmark: the bench shape (B=32,
L=319 = 256 image + 63 text tokens, two segments) and SURVEY C2 (B=32,
L=2048, one segment), 10 heads x 256, window 2048.  Device time per launch
(graph-captured) and MFMA TFLOP/s on the VISIBLE (query, key) pairs only
(4 * H * hd FLOP each: QK^T and PV under the segment / causal / window mask)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops


def timeit(fn, reps=10):
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
  H, hd, W = 10, 256, 2048
  for b, l, split in ((32, 319, 256), (32, 2048, 0), (1, 319, 256)):
    pos = torch.arange(l, dtype=torch.int32)[None].repeat(b, 1)
    if split:
      pos[:, split:] = torch.arange(l - split, dtype=torch.int32)
    pos = pos.to(dev)
    q = (torch.randn(b * l, H * hd, device=dev)).to(torch.bfloat16)
    k = (torch.randn(b * l, hd, device=dev)).to(torch.bfloat16)
    v = (torch.randn(b * l, hd, device=dev)).to(torch.bfloat16)
    seg, start = ops.ops.segment_info(pos)
    idx = torch.arange(l, device=dev)
    lo = torch.maximum(start.long(), idx - W)
    flops = float((idx - lo + 1).sum()) * 4 * H * hd
    us = timeit(lambda: ops.ops.local_attention(q, k, v, seg, start, b, l, H, hd, W))
    print(f"local attention B {b:2d} L {l:5d} split {split:3d}: {us:9.1f} us "
          f"{flops / us / 1e6:8.1f} TFLOP/s ({flops / us / 1e6 / 2500:.1%} of 2.5 PF, "
          f"{flops / 1e9:.1f} GFLOP visible)", flush=True)


if __name__ == "__main__":
  main()
