"""Run-to-run determinism of the attention kernels and the ViT towers: the
same inputs must give bit-identical outputs on every launch (no atomics in
these paths, fixed reduction orders).  An inline-asm VALU reading a fresh
MFMA result inside the hardware's wait-state window read stale
accumulators on some waves of some launches -- ~3 % of the ViT attention
outputs moved by one bf16 ulp between launches -- and no tolerance test saw
it; these tests do.
"""

import pytest
import torch

from cadence import common, ops, vision

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _same(outs, what):
  for i, o in enumerate(outs[1:], 1):
    assert torch.equal(o, outs[0]), f"{what}: launch {i} differs from launch 0"


@pytest.mark.parametrize("b,n,h,hd", [(32, 261, 16, 64), (32, 256, 16, 72),
                                      (4, 581, 16, 64), (4, 729, 16, 72),
                                      (32, 581, 16, 64), (32, 576, 16, 72)])
def test_vit_attention_deterministic(dev, b, n, h, hd):
  g = torch.Generator().manual_seed(3)
  qkv = torch.randn(b * n, 3 * h * hd, generator=g).to(BF).to(dev)
  _same([ops.ops.vit_attention(qkv, b, n, h, hd) for _ in range(8)],
        f"vit_attention N={n} hd={hd}")


@pytest.mark.parametrize("b,t", [(32, 319), (2, 2048)])
def test_griffin_attention_deterministic(dev, b, t):
  g = torch.Generator().manual_seed(5)
  h, hd = 10, 256
  q = torch.randn(b * t, h * hd, generator=g).to(BF).to(dev)
  k = torch.randn(b * t, hd, generator=g).to(BF).to(dev)
  v = torch.randn(b * t, hd, generator=g).to(BF).to(dev)
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  pos[:, 256:] -= 256                      # image segment + text segment
  seg, start = ops.ops.segment_info(pos.to(dev))
  _same([ops.ops.local_attention(q, k, v, seg, start, b, t, h, hd, 2048)
         for _ in range(6)], f"local attention B={b} T={t}")


def test_vit_towers_deterministic(dev):
  """Full-depth DINOv2 + SigLIP towers on two streams, three launches."""
  torch.manual_seed(0)
  cfg = common.VisionConfig(image_size=224)
  enc = vision.VisionEncoder(device=dev, config=cfg)
  px = torch.rand(2, 3, 224, 224, generator=torch.Generator().manual_seed(1)).to(dev)
  outs = []
  for _ in range(3):
    out = torch.zeros(2 * cfg.n_visual_tokens, cfg.feature_width, dtype=BF, device=dev)
    with torch.no_grad():
      enc.features_into(px, out)
    outs.append(out)
  _same(outs, "ViT features")
