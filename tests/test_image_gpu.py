"""GPU image preprocessing (cadence_resize_bicubic) vs Pillow.

The reference resizes each image on the host with torchvision Resize((S, S),
BICUBIC) on a PIL image + ToTensor (dino_siglip.py:12-16, 88-124, 148-151);
Pillow (the reference's own dependency) is the checker: bit-exact uint8
results, /255 in fp32.
"""

import numpy as np
import pytest
import torch

from oracle import griffin_ref as R

import cadence
from cadence import common, image_io

pytestmark = pytest.mark.gpu


def _images(rng, shapes):
  out = []
  for i, (h, w) in enumerate(shapes):
    if i % 2:
      yy, xx = np.mgrid[0:h, 0:w]
      a = np.stack([xx * 255 // max(w - 1, 1), yy * 255 // max(h - 1, 1),
                    (xx * 7 + yy * 3) % 256], -1).astype(np.uint8)
    else:
      a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    out.append(a)
  return out


@pytest.mark.parametrize("size", [224, 336, 384, 56])
def test_resize_ragged_batch_bitexact(dev, size):
  rng = np.random.default_rng(size)
  shapes = [(480, 640), (100, 150), (size, size), (1, 7), (2217, 1353),
            (50, 2000), (333, 517), (7, 1), (3, 6000)]   # > 5450 wide: unstaged rows
  imgs = _images(rng, shapes)
  got = image_io.resize_arrays(imgs, size, dev).cpu()
  assert got.shape == (len(imgs), 3, size, size)
  for i, a in enumerate(imgs):
    want = R.pil_resize_to_tensor(a, size)
    assert torch.equal(got[i], want), (shapes[i], size)
  # small images only: the coefficient tables fit in LDS (the batch above
  # takes the global-table path) and every column pass is LDS-staged
  small = [(480, 640), (300, 200), (size, size), (3, 5)]
  imgs = _images(rng, small)
  got = image_io.resize_arrays(imgs, size, dev).cpu()
  for i, a in enumerate(imgs):
    assert torch.equal(got[i], R.pil_resize_to_tensor(a, size)), (small[i], size)


def test_resize_rejects_bad_input(dev):
  with pytest.raises(ValueError):
    image_io.resize_arrays([np.zeros((4, 4), np.uint8)], 224, dev)
  with pytest.raises(ValueError):
    image_io.resize_arrays([], 224, dev)



def test_img_path_list_feeds_the_model(dev, tmp_path):
  """Griffin.forward(img_path=[...]) == forward(images=Pillow-resized pixels)."""
  from PIL import Image
  rng = np.random.default_rng(7)
  paths = []
  for i, (h, w) in enumerate([(90, 120), (64, 40)]):
    p = tmp_path / f"im{i}.png"
    Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(p)
    paths.append(str(p))
  dino = common.ViTConfig(name="dino", width=1024, depth=1, num_heads=16,
                          mlp_width=4096, class_token=True, reg_tokens=4,
                          layer_scale=True)
  sig = common.ViTConfig(name="siglip", width=1152, depth=1, num_heads=16,
                         mlp_width=4304, mean=common.SIGLIP_MEAN,
                         std=common.SIGLIP_STD)
  vis = common.VisionConfig(image_size=56, dino=dino, siglip=sig, feature_block=0)
  cfg = common.GriffinConfig(
      vocab_size=256, width=256, mlp_expanded_width=768, num_heads=4,
      block_types=(common.TemporalBlockType.RECURRENT,
                   common.TemporalBlockType.ATTENTION),
      embeddings_scale_by_sqrt_dim=True, attention_window_size=2048,
      logits_soft_cap=30.0)
  torch.manual_seed(0)
  m = cadence.Griffin(cfg, device=dev, dtype=torch.bfloat16, vision=vis)
  tok = torch.randint(3, 256, (2, 6), dtype=torch.int32, device=dev)
  pos = torch.arange(6, dtype=torch.int32, device=dev)[None].repeat(2, 1)
  px = torch.stack([R.pil_resize_to_tensor(image_io.decode_rgb(p), 56)
                    for p in paths]).to(dev)
  with torch.no_grad():
    a, _ = m(tok, pos, img_path=paths)
    b, _ = m(tok, pos, images=px)
    one, _ = m(tok, pos, img_path=paths[0])      # reference form: one image
    ref1, _ = m(tok, pos, images=px[:1].expand(2, -1, -1, -1).contiguous())
  assert torch.equal(a, b)
  assert torch.equal(one, ref1)
