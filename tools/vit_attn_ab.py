"""Lab A/B of the ViT attention kernels at one shape under engine masks
(cadence_gemm_set_engine bits, e.g. 15 = default, 31 = + bit 4): per mask the
kernel name the plan picks, HIP-event time over 20 launches (median of 5),
MFMA fraction of 2.5 PF, and whether the output equals the first mask's.
    python tools/vit_attn_ab.py B N H hd MASK [MASK ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import _lib, ops


def main():
  b, n, h, hd = (int(v) for v in sys.argv[1:5])
  masks = [int(v) for v in sys.argv[5:]]
  dev = torch.device("cuda")
  g = torch.Generator().manual_seed(0)
  qkv = torch.randn(b * n, 3 * h * hd, generator=g).to(torch.bfloat16).to(dev)
  lib = _lib.load()
  flop = 4.0 * n * n * hd * b * h
  ref = None
  for m in masks:
    prev = lib.cadence_gemm_set_engine(m)
    try:
      out = ops.ops.vit_attention(qkv, b, n, h, hd)
      torch.cuda.synchronize()
      same = ref is None or torch.equal(out, ref)
      if ref is None:
        ref = out.clone()
      ts = []
      for _ in range(5):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(20):
          ops.ops.vit_attention(qkv, b, n, h, hd)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20 * 1e3)
      ts.sort()
      us = ts[2]
      print(f"mask {m}: {us:.2f} us  {flop / us / 1e6 / 2500:.3f} of 2.5 PF  "
            f"equal to mask {masks[0]}: {same}", flush=True)
    finally:
      lib.cadence_gemm_set_engine(prev)


if __name__ == "__main__":
  main()
