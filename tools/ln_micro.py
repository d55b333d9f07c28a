"""ViT LayerNorm alone at the bench shape (B = 32, 224 px): DINO 8352 x 1024,
SigLIP 8192 x 1152 fp32 rows -> bf16; HBM GB/s of the algorithmic bytes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops
dev = torch.device("cuda", 0)
for rows, w in ((32 * 261, 1024), (32 * 256, 1152)):
  x = torch.randn(rows, w, device=dev)
  sc = torch.randn(w, device=dev).to(torch.bfloat16)
  b = torch.randn(w, device=dev).to(torch.bfloat16)
  fn = lambda: ops.ops.layernorm(x, sc, b, 1e-6)
  fn(); torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(20):
      fn()
  g.replay(); torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record(); g.replay(); e.record(); torch.cuda.synchronize()
  us = s.elapsed_time(e) / 20 * 1e3
  nb = rows * w * 6
  print(f"layernorm {rows}x{w}: {us:.1f} us  {nb / us / 1e3:.0f} GB/s", flush=True)
