"""RG-LRU scan microbenchmark (HBM-bound): the fused gated scan at the bench
shape (B=32, L=319 = 256 image + 63 prompt tokens, E=2560) and at SURVEY C2
(B=32, L=2048).  CADENCE_SCAN=lds|reg2|reg1 selects the engine (read once
per process).  Bytes are algorithmic: x, a, gate in + y out (bf16) per
element, positions, fp32 state in/out."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops


def main():
  dev = torch.device("cuda")
  reps = int(os.environ.get("REPS", "20"))
  mode = os.environ.get("CADENCE_SCAN", "lds")
  for b, l, e in ((32, 319, 2560), (32, 2048, 2560)):
    m = b * l
    x = torch.randn(m, e, device=dev).to(torch.bfloat16)
    a = torch.rand(m, e, device=dev).to(torch.bfloat16)
    yx = torch.randn(m, 2 * e, device=dev).to(torch.bfloat16)
    gate = yx[:, :e]
    pos = torch.arange(l, dtype=torch.int32, device=dev)[None].repeat(b, 1)
    h0 = torch.randn(b, e, device=dev)
    fn = lambda: ops.ops.rnn_scan(x, a, pos, h0, gate, b, l)
    fn(); torch.cuda.synchronize()
    s, t = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(reps):
      fn()
    t.record(); torch.cuda.synchronize()
    us = s.elapsed_time(t) / reps * 1e3
    nbytes = m * e * 8 + m * 4 + b * e * 8
    print(f"scan {mode:5s} B {b} L {l:5d} E {e}: {us:8.1f} us "
          f"{nbytes / us / 1e3:7.1f} GB/s ({nbytes / us / 1e3 / 8000:.1%} of 8 TB/s)",
          flush=True)


if __name__ == "__main__":
  main()
