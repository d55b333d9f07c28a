"""ViT tower cost at the bench shape (B = 32, 224 px): wall time of the two
towers on two streams vs back to back, the projector, and each tower GEMM
shape alone (TF/s of 2 M N K)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
from cadence import common, ops, vision  # noqa: E402

dev = torch.device("cuda", 0)
BF = torch.bfloat16


def timeit(fn, reps=10):
  fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


torch.manual_seed(0)
cfg = common.VisionConfig(image_size=224)
enc = vision.VisionEncoder(device=dev, config=cfg)
b = 32
px = torch.rand(b, 3, 224, 224, device=dev)
out = torch.empty(b * cfg.n_visual_tokens, cfg.feature_width, dtype=BF, device=dev)
with torch.no_grad():
  t2 = timeit(lambda: enc.features_into(px, out))
  td = timeit(lambda: enc.dino.features_into(px, out, 0, cfg.blocks_run))
  ts = timeit(lambda: enc.siglip.features_into(px, out, cfg.dino.width, cfg.blocks_run))
print(f"towers on two streams {t2:.0f} us; DINO alone {td:.0f} us, SigLIP alone {ts:.0f} us, "
      f"sum {td + ts:.0f} us", flush=True)

shapes = [("dino qkv", 32 * 261, 3072, 1024, 0), ("dino proj", 32 * 261, 1024, 1024, 0),
          ("dino fc1", 32 * 261, 4096, 1024, 1), ("dino fc2", 32 * 261, 1024, 4096, 0),
          ("sig qkv", 32 * 256, 3456, 1152, 0), ("sig proj", 32 * 256, 1152, 1152, 0),
          ("sig fc1", 32 * 256, 4352, 1152, 1), ("sig fc2", 32 * 256, 1152, 4352, 0)]
for name, m, n, k, act in shapes:
  a = (torch.rand(m, k, device=dev) * 2 - 1).to(BF)
  w = ((torch.rand(n, k, device=dev) * 2 - 1) / k ** .5).to(BF)
  o = torch.empty(m, n, device=dev, dtype=BF)
  us = timeit(lambda: ops.linear(a, w, act=act, out=o), 20)
  rows = ops._lib.load().cadence_gemm_tile_rows(m, n, k, 1)
  tiles = -(-m // rows) * -(-n // 256)
  print(f"{name:10s} {m}x{n}x{k} act{act}: {us:7.1f} us {2 * m * n * k / us / 1e6:7.1f} TF/s "
        f"({rows}-row tiles: {tiles})", flush=True)
