"""Lab A/B: prefill RG-LRU gates + scan as two kernels (rglru_gates_stream
then rnn_scan) vs the fused rglru_scan kernel at a shape (B, L; 10 blocks of
256), interleaved rounds in one process, HIP events; checks bitwise equality.
    python tools/rglru_fused_ab.py [B L]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops


def main():
  b = int(sys.argv[1]) if len(sys.argv) > 1 else 32
  t = int(sys.argv[2]) if len(sys.argv) > 2 else 319
  h, bw = 10, 256
  e = h * bw
  dev = torch.device("cuda")
  g = torch.Generator().manual_seed(0)
  yx = torch.randn(b * t, 2 * e, generator=g).to(torch.bfloat16).to(dev)
  x, gate = yx[:, e:], yx[:, :e]
  w = (torch.randn(h, 2 * bw, bw, generator=g) / 16).to(torch.bfloat16).to(dev)
  bx = (torch.randn(e, generator=g) * .3).to(torch.bfloat16).to(dev)
  ba = (torch.randn(e, generator=g) * .3).to(torch.bfloat16).to(dev)
  sp = torch.rand(e, generator=g).to(torch.bfloat16).to(dev)
  pos = torch.arange(t, dtype=torch.int32).repeat(b).to(dev)
  two = lambda: ops.ops.rnn_scan(*ops.ops.rglru_gates(x, w, bx, ba, sp, pos)[::-1], None, None, gate, b, t)
  fused = lambda: ops.ops.rglru_scan(x, w, bx, ba, sp, pos, None, gate, b, t)
  y0, h0 = two()
  y1, h1 = fused()
  print("bitwise", torch.equal(y0, y1) and torch.equal(h0, h1), flush=True)
  res = {"two": [], "fused": []}
  for _ in range(5):
    for name, fn in (("two", two), ("fused", fused)):
      s, en = torch.cuda.Event(True), torch.cuda.Event(True)
      s.record()
      for _ in range(20):
        fn()
      en.record()
      torch.cuda.synchronize()
      res[name].append(s.elapsed_time(en) / 20 * 1e3)
  for k, v in res.items():
    v = sorted(v)
    print(f"B={b} L={t} {k:6s} median {v[len(v)//2]:.1f} us  min {v[0]:.1f} us", flush=True)


if __name__ == "__main__":
  main()
