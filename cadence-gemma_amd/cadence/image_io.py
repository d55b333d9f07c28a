"""Host-side image loading for the `img_path` API of the reference.

Reference: `pil_loader` + timm eval transforms (dino_siglip.py:12-16,
88-124, 148-151): RGB convert, Resize((S, S), bicubic), CenterCrop(S) (a
no-op after the square resize), ToTensor.  The per-encoder Normalize is
folded into the im2col kernel on the GPU.  Batched synthetic inputs bypass
this module entirely (`Griffin.forward(images=...)`).
"""

from __future__ import annotations

import numpy as np
import torch


def load_image(path: str, size: int) -> torch.Tensor:
  from PIL import Image  # host dependency of the reference too
  with open(path, "rb") as f:
    img = Image.open(f).convert("RGB")
  img = img.resize((size, size), Image.BICUBIC)
  arr = np.asarray(img, dtype=np.float32) / 255.0          # [S, S, 3]
  return torch.from_numpy(arr).permute(2, 0, 1).contiguous()
