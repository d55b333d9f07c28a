"""Does a decode GEMV read its weights faster when they were just read by
another kernel (Infinity Cache / MALL residency)?  The gated up-projection
GEMV (M = 32, 2F = 15360, K = 2560: 78.6 MB of fragment-packed weights)
timed (1) cold: after streaming a 1 GiB buffer through the caches; (2) warm:
the same weights read by a torch reduction first; (3) concurrent: a torch
reduction of the NEXT layer's weights on a side stream while this GEMV
runs (does the prefetch slow the GEMV, and is the next one then warm?).
usage: python tools/mall_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import ops  # noqa: E402

BF = torch.bfloat16


def main():
  dev = torch.device("cuda")
  M, F, K = 32, 7680, 2560
  layers = 6
  ws = [(torch.randn(2 * F, K, device=dev) * 0.02).to(BF) for _ in range(layers)]
  bg = torch.zeros(F, device=dev, dtype=BF)
  bu = torch.zeros(F, device=dev, dtype=BF)
  x = torch.randn(M, K, device=dev).to(BF)
  for w in ws:
    ops.gated_gelu(x, w, bg, bu)          # build the packed decode copies
  wd = [ops.decode_weight(w) for w in ws]
  flush = torch.empty(1 << 28, device=dev, dtype=torch.float32)   # 1 GiB
  side = torch.cuda.Stream()
  torch.cuda.synchronize()

  def ev():
    return torch.cuda.Event(enable_timing=True)

  def gemv(i):
    return ops.gated_gelu(x, ws[i], bg, bu)

  res = {"cold": [], "warm": [], "with_prefetch": [], "after_prefetch": []}
  for rep in range(5):
    for i in range(layers - 1):
      flush.add_(1.0)
      torch.cuda.synchronize()
      a, b = ev(), ev()
      a.record(); gemv(i); b.record()
      torch.cuda.synchronize()
      res["cold"].append(a.elapsed_time(b) * 1e3)
      flush.add_(1.0)
      wd[i].view(torch.int32).sum()
      torch.cuda.synchronize()
      a, b = ev(), ev()
      a.record(); gemv(i); b.record()
      torch.cuda.synchronize()
      res["warm"].append(a.elapsed_time(b) * 1e3)
      # layer i with layer i + 1's weights read on the side stream meanwhile
      flush.add_(1.0)
      torch.cuda.synchronize()
      a, b, c, d = ev(), ev(), ev(), ev()
      a.record()
      side.wait_stream(torch.cuda.current_stream())
      with torch.cuda.stream(side):
        wd[i + 1].view(torch.int32).sum()
      gemv(i)
      b.record()
      torch.cuda.current_stream().wait_stream(side)
      c.record(); gemv(i + 1); d.record()
      torch.cuda.synchronize()
      res["with_prefetch"].append(a.elapsed_time(b) * 1e3)
      res["after_prefetch"].append(c.elapsed_time(d) * 1e3)
  nbytes = 2 * F * K * 2
  for k, v in res.items():
    v = sorted(v)
    med = v[len(v) // 2]
    print(f"{k:15s} median {med:7.2f} us  ({nbytes / med / 1e3:6.0f} GB/s)  min {v[0]:.2f}",
          flush=True)


if __name__ == "__main__":
  main()
