"""RG-LRU scan microbenchmark (HBM-bound): the fused gated scan at the bench
shape (B=32, L=319 = 256 image + 63 prompt tokens, E=2560), SURVEY C2
(B=32, L=2048) and the small-batch shapes the chunked form serves (C3:
B=1, L=319; B=1, L=2048; B=4, L=319).  Each shape is timed through the op
(chunked form where the plan picks it) and through the C-ABI with no
workspace (the one-lane-per-sequence kernel).  Bytes are algorithmic:
x, a, gate in + y out (bf16) per element, positions, fp32 state in/out."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops, _lib


def timeit(fn, reps):
  """GPU time per call: `reps` calls captured in one hipGraph and replayed
  (no host launch overhead between them)."""
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
  s.record()
  g.replay()
  t.record(); torch.cuda.synchronize()
  return s.elapsed_time(t) / reps * 1e3


def main():
  dev = torch.device("cuda")
  reps = int(os.environ.get("REPS", "20"))
  lib = _lib.load()
  for b, l, e in ((1, 319, 2560), (1, 2048, 2560), (4, 319, 2560),
                  (32, 319, 2560), (32, 2048, 2560)):
    m = b * l
    x = torch.randn(m, e, device=dev).to(torch.bfloat16)
    a = torch.rand(m, e, device=dev).to(torch.bfloat16)
    yx = torch.randn(m, 2 * e, device=dev).to(torch.bfloat16)
    gate = yx[:, :e]
    pos = torch.arange(l, dtype=torch.int32, device=dev)[None].repeat(b, 1)
    h0 = torch.randn(b, e, device=dev)
    out = torch.empty(m, e, device=dev, dtype=torch.bfloat16)
    hl = torch.empty(b, e, device=dev)
    seq = lambda: lib.cadence_rnn_scan(
        x.data_ptr(), e, a.data_ptr(), e, pos.data_ptr(), h0.data_ptr(),
        gate.data_ptr(), 2 * e, out.data_ptr(), e, hl.data_ptr(), b, l, e,
        None, 0, torch.cuda.current_stream().cuda_stream)
    op = lambda: ops.ops.rnn_scan(x, a, pos, h0, gate, b, l)
    chunked = lib.cadence_rnn_scan_workspace_bytes(b, l, e) > 0
    nbytes = m * e * 8 + m * 4 + b * e * 8
    for name, fn in (("op" + ("(chunked)" if chunked else ""), op),
                     ("sequential", seq)):
      us = timeit(fn, reps)
      print(f"scan B {b:2d} L {l:5d} E {e} {name:14s}: {us:8.1f} us "
            f"{nbytes / us / 1e3:7.1f} GB/s ({nbytes / us / 1e3 / 8000:.1%} "
            f"of 8 TB/s)", flush=True)


if __name__ == "__main__":
  main()
