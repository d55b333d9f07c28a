"""Graph-timed decode attention (one token step, B = 32, 10 heads, hd 256,
window 2048) at several context lengths: the bench's (~320-350 keys), 1k,
and a wrapped 2048-slot ring (C2).  Each replay advances the ring by one
token (in place), as in the decode graph.
usage: python tools/decode_attn_micro.py"""

import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cadence-gemma_amd"))
from cadence import ops  # noqa: E402


def main():
  dev = torch.device("cuda", 0)
  B, H, hd, W = 32, 10, 256, 2048
  g = torch.Generator(device=dev).manual_seed(0)
  ck = torch.randn(B, W, hd, device=dev, generator=g).to(torch.bfloat16)
  cv = torch.randn(B, W, hd, device=dev, generator=g).to(torch.bfloat16)
  q = torch.randn(B, H * hd, device=dev, generator=g).to(torch.bfloat16)
  kn = torch.randn(B, hd, device=dev, generator=g).to(torch.bfloat16)
  vn = torch.randn(B, hd, device=dev, generator=g).to(torch.bfloat16)
  reps = 20
  for ctx in (64, 128, 320, 1000, 2100):
    nt = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    # warm-up on the capture stream: the split combine's arrival counters
    # are per stream and must exist before capture (as in the sampler)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
      for _ in range(2):
        ops.ops.local_attention_decode_(q, kn, vn, ck, cv, nt, H)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
      for _ in range(reps):
        ops.ops.local_attention_decode_(q, kn, vn, ck, cv, nt, H)
    best = 1e9
    for _ in range(5):
      nt.fill_(ctx)
      a = torch.cuda.Event(enable_timing=True)
      b = torch.cuda.Event(enable_timing=True)
      a.record()
      graph.replay()
      b.record()
      b.synchronize()
      best = min(best, a.elapsed_time(b) * 1e3 / reps)
    kv = B * min(ctx + reps, W) * hd * 2 * 2
    print(f"ctx {ctx:5d}: {best:7.2f} us per step  ({kv / (best * 1e-6) / 1e9:7.1f} GB/s "
          f"of K/V)", flush=True)


if __name__ == "__main__":
  main()
