"""Image loading for the `img_path` API of the reference, resized on the GPU.

Reference: `pil_loader` + the timm eval transforms of both encoders
(dino_siglip.py:12-16, 88-124, 148-151): RGB convert, Resize((S, S),
bicubic), CenterCrop(S) (a no-op after the square resize), ToTensor, then the
per-encoder Normalize.  Both encoders resize the same image to the same size
with the same filter, so one resize serves both.

Here the host only decodes (JPEG/PNG -> uint8 HWC, Pillow, as the reference
does; a thread pool decodes a list of paths in parallel) and packs the ragged
batch into one pinned buffer.  The bicubic resize + ToTensor run on the GPU
(`cadence_resize_bicubic`, bit-exact with Pillow's resampler) and the
Normalize is folded into the patch extraction (`cadence_im2col_normalize`).
"""

from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import Sequence

import numpy as np
import torch

from . import ops


def decode_rgb(path: str) -> np.ndarray:
  """pil_loader (dino_siglip.py:12-16): open, convert('RGB') -> [H, W, 3] u8."""
  from PIL import Image  # host dependency of the reference too
  with open(path, "rb") as f:
    img = Image.open(f)
    return np.asarray(img.convert("RGB"), dtype=np.uint8)


def resize_arrays(arrays: Sequence[np.ndarray], size: int,
                  device) -> torch.Tensor:
  """Ragged uint8 HWC RGB images -> [B, 3, size, size] fp32 in [0, 1] on
  `device` (Resize((size, size), BICUBIC) + ToTensor, Pillow-exact)."""
  if not arrays:
    raise ValueError("no images")
  meta = np.zeros((len(arrays), 4), dtype=np.int64)
  off = tmp = 0
  ks = 5
  for i, a in enumerate(arrays):
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3 or min(a.shape[:2]) < 1:
      raise ValueError(f"image {i}: want uint8 [H, W, 3], got {a.dtype} {a.shape}")
    h, w = a.shape[:2]
    meta[i] = (off, h, w, tmp)
    off += h * w * 3
    tmp += h * size * 3
    ks = max(ks, ops.resize_taps(h, size), ops.resize_taps(w, size))
  packed = torch.empty(off, dtype=torch.uint8, pin_memory=True)
  view = packed.numpy()
  for i, a in enumerate(arrays):
    view[meta[i, 0]:meta[i, 0] + a.size] = np.ascontiguousarray(a).reshape(-1)
  dev_images = packed.to(device, non_blocking=True)
  dev_meta = torch.from_numpy(meta).pin_memory().to(device, non_blocking=True)
  max_h, max_w = int(meta[:, 1].max()), int(meta[:, 2].max())
  return torch.ops.cadence.resize_bicubic(dev_images, dev_meta, size, ks, max_h,
                                          max_w, tmp)


def load_images(paths: str | Sequence[str], size: int, device,
                workers: int = 8) -> torch.Tensor:
  """img_path (or a list of them) -> [B, 3, size, size] fp32 pixels on device."""
  if isinstance(paths, str):
    paths = [paths]
  if len(paths) == 1:
    arrays = [decode_rgb(paths[0])]
  else:
    with ThreadPoolExecutor(max_workers=min(workers, len(paths))) as pool:
      arrays = list(pool.map(decode_rgb, paths))
  return resize_arrays(arrays, size, device)
