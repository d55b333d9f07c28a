"""Probe: (1) do forked branches of a captured hipGraph run concurrently;
(2) how much faster is a decode GEMV whose weights are Infinity-Cache
resident (warm) than one streaming them from HBM (cold); (3) does a side-
stream read of the next weights ahead of the GEMV make it warm.
usage: python tools/prefetch_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cadence-gemma_amd"))
from cadence import ops  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)


def timed(fn, n=20):
  s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  fn()
  torch.cuda.synchronize()
  s.record()
  for _ in range(n):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / n * 1000.0


# (1) graph branch concurrency
main = torch.cuda.Stream()
side = torch.cuda.Stream()
cyc = 200000
for fork in (False, True):
  g = torch.cuda.CUDAGraph()
  with torch.cuda.stream(main):
    torch.cuda._sleep(10)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=main):
      if fork:
        side.wait_stream(main)
        with torch.cuda.stream(side):
          torch.cuda._sleep(cyc)
      torch.cuda._sleep(cyc)
      if fork:
        main.wait_stream(side)
  t = timed(g.replay, 10)
  print(f"graph sleep x{'2 forked' if fork else '1'}: {t:.1f} us", flush=True)
with torch.cuda.stream(main):
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=main):
    torch.cuda._sleep(cyc)
    torch.cuda._sleep(cyc)
  print(f"graph sleep x2 serial: {timed(g.replay, 10):.1f} us", flush=True)

# (2) cold vs warm gated GEMV at the decode shape
M, F, K = 32, 7680, 2560
x = ops.pack_rows(torch.randn(M, K, device=dev).to(torch.bfloat16))
ws = [ops.pack_decode((torch.randn(2 * F, K, device=dev) * K ** -0.5).to(torch.bfloat16))
      for _ in range(8)]
bg = torch.zeros(F, dtype=torch.bfloat16, device=dev)
bu = torch.zeros(F, dtype=torch.bfloat16, device=dev)
it = iter(range(10 ** 9))


def cold():
  ops.ops.gated_gelu(x.data, ws[next(it) % 8], bg, bu, True, M, True)


def warm():
  ops.ops.gated_gelu(x.data, ws[0], bg, bu, True, M, True)


print(f"gated GEMV cold (8 weight sets, 630 MB): {timed(cold, 40):.1f} us", flush=True)
print(f"gated GEMV warm (same 79 MB): {timed(warm, 40):.1f} us", flush=True)

# (3) side-stream prefetch of the next weight set while a decode-like chain
# of small kernels runs on the main stream
sink = torch.empty(8, device=dev)
small = torch.randn(32, 2560, device=dev)


def chain_then_gemv(prefetch: bool, i: int):
  nxt = ws[i % 8]
  if prefetch:
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
      sink[0] = nxt.view(torch.int16).amax().float()
  for _ in range(6):
    torch.cuda._sleep(3000)     # ~latency-bound kernels (attention, gates, ...)
  ops.ops.gated_gelu(x.data, nxt, bg, bu, True, M, True)
  if prefetch:
    torch.cuda.current_stream().wait_stream(side)


for pf in (False, True):
  cnt = iter(range(10 ** 9))
  t = timed(lambda: chain_then_gemv(pf, next(cnt)), 40)
  print(f"chain + cold GEMV, prefetch={pf}: {t:.1f} us", flush=True)
