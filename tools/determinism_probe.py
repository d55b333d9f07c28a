"""Run-to-run determinism of the ViT path: the same pixels through the
full-depth towers several times, (a) one stream (towers back to back), (b)
the two-stream form, (c) single kernels (ViT attention, the prefill GEMM, the
ViT LayerNorm) repeated on fixed inputs.  Prints the max abs difference of
every repeat against the first."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
from cadence import common, ops, vision  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
cfg = common.VisionConfig(image_size=224)
enc = vision.VisionEncoder(device=dev, config=cfg)
b = int(os.environ.get("B", "2"))
px = torch.rand(b, 3, 224, 224, device=dev)
nv = cfg.n_visual_tokens


def run(two):
  out = torch.zeros(b * nv, cfg.feature_width, dtype=torch.bfloat16, device=dev)
  with torch.no_grad():
    if two:
      enc.features_into(px, out)
    else:
      enc.dino.features_into(px, out, 0, cfg.blocks_run)
      enc.siglip.features_into(px, out, cfg.dino.width, cfg.blocks_run)
  torch.cuda.synchronize()
  return out


def report(name, outs):
  d = [float((o.float() - outs[0].float()).abs().max()) for o in outs[1:]]
  print(f"{name:40s} max |diff| vs first: {d}", flush=True)


report("one stream", [run(False) for _ in range(4)])
report("two streams", [run(True) for _ in range(4)])
ref1 = run(False)
report("one stream vs two streams", [ref1, run(True), run(True)])

# single kernels
n, h, hd = 261, 16, 64
qkv = (torch.randn(b * n, 3 * h * hd, device=dev)).to(torch.bfloat16)
report("vit_attention hd64", [ops.ops.vit_attention(qkv, b, n, h, hd) for _ in range(6)])
qkv72 = (torch.randn(b * 256, 3 * 16 * 72, device=dev)).to(torch.bfloat16)
report("vit_attention hd72", [ops.ops.vit_attention(qkv72, b, 256, 16, 72) for _ in range(6)])
for m, nn_, k in ((522, 3072, 1024), (522, 4096, 1024), (10208, 15360, 2560), (2 * 319, 2560, 7680)):
  a = torch.randn(m, k, device=dev).to(torch.bfloat16)
  w = (torch.randn(nn_, k, device=dev) * k ** -0.5).to(torch.bfloat16)
  report(f"gemm {m}x{nn_}x{k}", [ops.linear(a, w) for _ in range(6)])
