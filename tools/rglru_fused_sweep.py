"""Fused prefill RG-LRU (rglru_scan_fused_kernel) time against the batch at
one length: how the (sequence, 128-channel) workgroup count fills the
resident slots (B * 20 workgroups, 2 per CU).  HIP events, 20 launches.
    python tools/rglru_fused_sweep.py L B [B ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops


def main():
  t = int(sys.argv[1])
  h, bw = 10, 256
  e = h * bw
  dev = torch.device("cuda")
  for b in [int(v) for v in sys.argv[2:]]:
    g = torch.Generator().manual_seed(0)
    yx = torch.randn(b * t, 2 * e, generator=g).to(torch.bfloat16).to(dev)
    x, gate = yx[:, e:], yx[:, :e]
    w = (torch.randn(h, 2 * bw, bw, generator=g) / 16).to(torch.bfloat16).to(dev)
    bx = (torch.randn(e, generator=g) * .3).to(torch.bfloat16).to(dev)
    ba = (torch.randn(e, generator=g) * .3).to(torch.bfloat16).to(dev)
    sp = torch.rand(e, generator=g).to(torch.bfloat16).to(dev)
    pos = torch.arange(t, dtype=torch.int32).repeat(b).to(dev)
    fn = lambda: ops.ops.rglru_scan(x, w, bx, ba, sp, pos, None, gate, b, t)
    fn()
    ts = []
    for _ in range(5):
      s, en = torch.cuda.Event(True), torch.cuda.Event(True)
      s.record()
      for _ in range(20):
        fn()
      en.record()
      torch.cuda.synchronize()
      ts.append(s.elapsed_time(en) / 20 * 1e3)
    ts.sort()
    us = ts[len(ts) // 2]
    print(f"B={b} L={t} workgroups {b * 20}: {us:.1f} us, {us / b:.2f} us per sequence",
          flush=True)


if __name__ == "__main__":
  main()
