"""Prefill norm kernels alone at the bench shapes, HIP events over REPS
launches: the ViT LayerNorm (fp32 rows in, bf16 out) at DINO / SigLIP 224 px
B = 32 and the Griffin RMSNorm (bf16 in / out) at B = 32 x 319 rows; prints
us and the fraction of 8 TB/s for the algorithmic bytes.
    python tools/norm_one.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops


def timed(fn, reps=50):
  fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  dev = torch.device("cuda")
  for m, d in ((32 * 261, 1024), (32 * 256, 1152)):
    x = torch.randn(m, d, device=dev)
    w = torch.randn(d, device=dev).to(torch.bfloat16)
    b = torch.randn(d, device=dev).to(torch.bfloat16)
    us = timed(lambda: ops.ops.layernorm(x, w, b, 1e-6))
    nb = m * d * (4 + 2)
    print(f"layernorm M={m} D={d}: {us:.2f} us  {nb / us / 1e3 / 8000:.3f} of 8 TB/s", flush=True)
  m, d = 32 * 319, 2560
  x = torch.randn(m, d, device=dev).to(torch.bfloat16)
  sc = torch.randn(d, device=dev).to(torch.bfloat16)
  us = timed(lambda: ops.rmsnorm(x, sc, 1e-6))
  nb = m * d * 4
  print(f"rmsnorm M={m} D={d}: {us:.2f} us  {nb / us / 1e3 / 8000:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
  main()
