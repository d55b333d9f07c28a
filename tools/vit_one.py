"""One ViT attention shape on the shipped plan, 30 launches (for rocprofv3
PMC passes).  env SHAPE=dino224|sig224|dino336|sig336, ENGINE=<bits>."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import _lib, ops  # noqa: E402

SHAPES = {"dino224": (261, 16, 64), "sig224": (256, 16, 72),
          "dino336": (581, 16, 64), "sig336": (576, 16, 72)}
n, h, hd = SHAPES[os.environ.get("SHAPE", "dino336")]
if "ENGINE" in os.environ:
  _lib.load().cadence_gemm_set_engine(int(os.environ["ENGINE"]))
b = 32
qkv = torch.randn(b * n, 3 * h * hd, device="cuda").to(torch.bfloat16)
for _ in range(30):
  ops.ops.vit_attention(qkv, b, n, h, hd)
torch.cuda.synchronize()
s, e = torch.cuda.Event(True), torch.cuda.Event(True)
s.record()
for _ in range(20):
  ops.ops.vit_attention(qkv, b, n, h, hd)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / 20 * 1e3
print(f"{os.environ.get('SHAPE', 'dino336')}: {us:.2f} us  {4.0 * b * h * n * n * hd / us / 1e6 / 2500:.3f} of 2.5 PF")
