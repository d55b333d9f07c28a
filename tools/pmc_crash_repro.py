"""Minimal reproducer of the rocprofv3 PMC-mode crash.

Plain PyTorch only -- no cadence kernel, no cadence library loaded -- in the
shape of the sampler's two-lane pipeline (cadence/sampler.py generate_many):
two lane streams; per micro-batch on its lane: a host tensor staged through
pinned memory and copied asynchronously (sampler._to_device), a few eager
kernels standing in for the prefill, then replays of a hipGraph captured
once per lane (the decode graph), then an event recorded on the lane
(the continuous lanes' hand-over).  Modes switch those pieces off one by
one:

  full      pinned async copies + graph replays + lane events
  nocopy    blocking pageable copies instead of the pinned async ones
  nograph   eager kernels instead of the graph replays
  noevent   no lane events (the caller's stream joins the lanes at the end)
  deep      full, with a 128-kernel captured graph per lane (the decode
            step's shape: ~130 short launches per replay), 32 replays per
            micro-batch
  pace      full + the round-4 host pacing: before queueing on a lane the host
            synchronizes that lane's previous timing event (recorded after
            its "prefill", while the other lane replays its graph)

    python tools/pmc_crash_repro.py MODE [ITERS]

Run it under `rocprofv3 --pmc FETCH_SIZE -- python3 tools/pmc_crash_repro.py
full` (tools/pmc_crash_repro.sh) and without the profiler: a crash under the
profiler only, in plain torch code, is the profiler's.
"""

import faulthandler
import sys

import torch

faulthandler.enable()


def main():
  mode = sys.argv[1] if len(sys.argv) > 1 else "full"
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  lanes = [torch.cuda.Stream() for _ in range(2)]
  w = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
  graphs, statics = [], []
  for ln in lanes:                       # one captured "decode step" per lane
    x = torch.randn(32, 1024, device=dev, dtype=torch.bfloat16)
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    def body():
      if mode == "deep":                 # ~130 short kernels, like a decode step
        for _ in range(64):
          x.mul_(0.999).add_(1e-3)
      y = torch.tanh(x @ w)
      x.copy_(y)
    with torch.cuda.stream(cap):
      body()                             # warm-up
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g, stream=cap):
        body()
    torch.cuda.current_stream().wait_stream(cap)
    graphs.append(g)
    statics.append(x)
  cur = torch.cuda.current_stream()
  for ln in lanes:
    ln.wait_stream(cur)
  ready = [None, None]
  pace = [None, None]
  outs = []
  for i in range(iters):
    j = i % 2
    ln = lanes[j]
    if mode == "pace" and pace[j] is not None:
      pace[j].synchronize()
    with torch.cuda.stream(ln):
      host = torch.arange(64, dtype=torch.int32) + i
      if mode == "nocopy":
        pos = host.to(dev)
      else:
        pos = host.pin_memory().to(dev, non_blocking=True)
      a = torch.randn(256, 1024, device=dev, dtype=torch.bfloat16)
      b = (a @ w).float().sum(1) + pos.float().sum()      # "prefill"
      if mode == "pace":
        pace[j] = torch.cuda.Event(enable_timing=True)
        pace[j].record(ln)
      for _ in range(32 if mode == "deep" else 8):        # "decode"
        if mode == "nograph":
          statics[j].copy_(torch.tanh(statics[j] @ w))
        else:
          graphs[j].replay()
      outs.append(b[:1] + statics[j].float().sum())
      if mode != "noevent":
        e = torch.cuda.Event()
        e.record(ln)
        ready[j] = e
  if mode != "noevent":
    for e in ready:
      cur.wait_event(e)
  for ln in lanes:
    cur.wait_stream(ln)
  torch.cuda.synchronize()
  print(f"pmc_crash_repro {mode}: ok, {iters} micro-batches, "
        f"checksum {float(torch.cat(outs).sum()):.4e}", flush=True)


if __name__ == "__main__":
  main()
