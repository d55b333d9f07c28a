"""Generates the golden fixtures under tests/golden/ (test infrastructure).

The reference commits no tensor fixtures and its Python cannot be run here
(import denied), so these vectors come from the CPU oracle
(oracle/griffin_ref.py), which is itself pinned by the reference's own KATs
(tests/test_oracle_kats.py).  They freeze the oracle's outputs so that
  * a later change to the oracle that alters its arithmetic is caught
    (tests/test_golden.py, CPU), and
  * the HIP path is checked against fixed vectors that do not depend on
    re-running the oracle on the GPU host (tests/test_golden.py, gpu).

Inputs are data (seeded), stored with the outputs.  Model weights are not
stored: `golden_params` rebuilds them from a seed on the CPU (torch's CPU
generator is deterministic for a given torch version) and the fixture holds
a float64 checksum per tensor so a drift in that rebuild fails loudly.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.safetensors
"""

from __future__ import annotations

import os
import sys

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for _p in (os.path.join(ROOT, "cadence-gemma_amd"), ROOT):
  if _p not in sys.path:
    sys.path.insert(0, _p)

from cadence import common  # noqa: E402
from oracle import griffin_ref as R  # noqa: E402

BF = torch.bfloat16
RA = common.TemporalBlockType


def two_doc_positions(b, t, split):
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  pos[:, split:] = torch.arange(t - split, dtype=torch.int32)
  return pos


def text_config():
  # Reference grid style (recurrentgemma/torch/modules_test.py): R, A, R
  # with a window shorter than the sequence so the window mask matters.
  return common.GriffinConfig(
      vocab_size=512, width=256, mlp_expanded_width=768, num_heads=4,
      block_types=(RA.RECURRENT, RA.ATTENTION, RA.RECURRENT),
      embeddings_scale_by_sqrt_dim=True, attention_window_size=24,
      logits_soft_cap=30.0)


def tiny_vision():
  dino = common.ViTConfig(name="dino", width=1024, depth=2, num_heads=16,
                          mlp_width=4096, class_token=True, reg_tokens=4,
                          layer_scale=True)
  sig = common.ViTConfig(name="siglip", width=1152, depth=2, num_heads=16,
                         mlp_width=4304, mean=common.SIGLIP_MEAN,
                         std=common.SIGLIP_STD)
  return common.VisionConfig(image_size=56, dino=dino, siglip=sig,
                             feature_block=1)


def golden_params(cfg, vision=None, seed=0):
  """CPU-initialised weights (the reference init recipes, as the model
  builds them), then every 1-D norm/bias/LayerScale perturbed so no path is
  an identity.  Returns a name -> bf16 CPU tensor dict (state-dict keys)."""
  import cadence
  torch.manual_seed(seed)
  m = cadence.Griffin(cfg, dtype=BF, vision=vision)
  g = torch.Generator().manual_seed(seed + 1)
  p = {}
  for k, v in m.state_dict().items():
    v = v.detach().clone()
    if k.endswith((".scale", ".bias", ".b", ".gamma")):
      v = (torch.randn(v.shape, generator=g) * 0.1).to(v.dtype) + (
          0.5 if k.endswith(".gamma") else 0.0)
    p[k] = v
  return p


def checksums(p):
  keys = sorted(p)
  return keys, torch.tensor([p[k].double().sum().item() for k in keys],
                            dtype=torch.float64)


def kernels():
  g = torch.Generator().manual_seed(20260301)
  out = {}
  # rnn_scan (layers.py:145-199): ragged T, resets mid-sequence, with h0
  b, t, e = 3, 67, 96
  x = torch.randn(b, t, e, generator=g).to(BF)
  a = torch.rand(b, t, e, generator=g).to(BF)
  reset = torch.rand(b, t, generator=g) < 0.07
  reset[:, 0] = True
  h0 = torch.randn(b, e, generator=g)
  y, h = R.rnn_scan(x, a, reset, h0)
  y0, h_0 = R.rnn_scan(x, a, reset, None)
  out.update({"scan.x": x, "scan.a": a, "scan.reset": reset.to(torch.uint8),
              "scan.h0": h0, "scan.y": y, "scan.h_last": h,
              "scan.y_noh0": y0, "scan.h_last_noh0": h_0})
  # scan, T == 1 decode branch (layers.py:175-182)
  x1 = torch.randn(4, 1, e, generator=g).to(BF)
  a1 = torch.rand(4, 1, e, generator=g).to(BF)
  r1 = torch.zeros(4, 1, dtype=torch.bool)
  h01 = torch.randn(4, e, generator=g)
  y1, hl1 = R.rnn_scan(x1, a1, r1, h01)
  out.update({"scan1.x": x1, "scan1.a": a1, "scan1.h0": h01, "scan1.y": y1,
              "scan1.h_last": hl1})
  # Conv1D prefill, two documents, both mask modes (layers.py:457-633)
  b, t, e = 2, 41, 128
  x = torch.randn(b, t, e, generator=g).to(BF)
  w = (torch.randn(4, e, generator=g) * 0.5).to(BF)
  bias = (torch.randn(e, generator=g) * 0.1).to(BF)
  pos = two_doc_positions(b, t, 13)
  out.update({"conv.x": x, "conv.w": w, "conv.b": bias, "conv.pos": pos})
  for compat in (True, False):
    yc, cc = R.conv1d(x, pos, w, bias, None, compat=compat)
    out[f"conv.y_compat{int(compat)}"] = yc
    out[f"conv.cache_compat{int(compat)}"] = cc
  # Conv1D decode step from a cache
  xd = torch.randn(b, 1, e, generator=g).to(BF)
  cd = torch.randn(b, 3, e, generator=g).to(BF)
  yd, cd2 = R.conv1d(xd, torch.full((b, 1), 9, dtype=torch.int32), w, bias, cd)
  out.update({"convd.x": xd, "convd.cache": cd, "convd.y": yd,
              "convd.cache_out": cd2})
  # RMSNorm (layers.py:70-78), wide rows
  xr = (torch.randn(9, 2560, generator=g) * 3).to(BF)
  sr = (torch.randn(2560, generator=g) * 0.2).to(BF)
  out.update({"rms.x": xr, "rms.scale": sr, "rms.y": R.rms_norm(xr, sr)})
  return out


def text_model():
  cfg = text_config()
  p = golden_params(cfg, seed=31)
  g = torch.Generator().manual_seed(32)
  b, t, steps = 2, 40, 6
  tok = torch.randint(3, cfg.vocab_size, (b, t), generator=g, dtype=torch.int32)
  tok[:, 0] = 2
  pos = two_doc_positions(b, t, 17)
  logits, _ = R.griffin_forward(p, cfg, tok.long(), pos)
  gtok, glog = R.greedy_sample(p, cfg, tok.long(), steps)
  keys, sums = checksums(p)
  return {"text.tokens": tok, "text.pos": pos, "text.logits": logits,
          "text.greedy_tokens": gtok.to(torch.int32),
          "text.greedy_logits": glog, "text.param_sums": sums}, keys


def mm_model():
  cfg = text_config()
  vis = tiny_vision()
  p = golden_params(cfg, vision=vis, seed=41)
  g = torch.Generator().manual_seed(42)
  b, t = 2, 12
  px = torch.rand(b, 3, 56, 56, generator=g)
  tok = torch.randint(3, cfg.vocab_size, (b, t), generator=g, dtype=torch.int32)
  tok[:, 0] = 2
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  feats = R.vision_encoder(px, p, vis)
  img = R.projector(feats, p)
  logits, _ = R.griffin_forward(p, cfg, tok.long(), pos, image_tokens=img)
  keys, sums = checksums(p)
  return {"mm.pixels": px, "mm.tokens": tok, "mm.pos": pos,
          "mm.features": feats.float(), "mm.image_tokens": img,
          "mm.logits": logits, "mm.param_sums": sums}, keys


IMAGES = ("car2.jpg", "german.jpg")   # recurrentgemma/vit/img_tests/ (data files)


def images():
  """pil_loader + Resize((S, S), BICUBIC) of two of the reference's own test
  images (dino_siglip.py:12-16, 88-124), expected uint8 outputs from Pillow."""
  import numpy as np
  from PIL import Image
  out = {}
  for name in IMAGES:
    with open(os.path.join(HERE, "images", name), "rb") as f:
      img = Image.open(f).convert("RGB")
    arr = np.asarray(img)
    out[f"{name}.decoded_sum"] = torch.tensor([int(arr.astype(np.int64).sum())])
    out[f"{name}.hw"] = torch.tensor(arr.shape[:2])
    for size in (224, 336):
      out[f"{name}.{size}"] = torch.from_numpy(
          np.array(img.resize((size, size), Image.BICUBIC), dtype=np.uint8))
  return out


def main():
  torch.set_num_threads(min(8, os.cpu_count() or 1))
  save_file({k: v.contiguous() for k, v in kernels().items()},
            os.path.join(HERE, "kernels.safetensors"))
  t, tkeys = text_model()
  save_file({k: v.contiguous() for k, v in t.items()},
            os.path.join(HERE, "text_model.safetensors"),
            metadata={"param_keys": ",".join(tkeys)})
  m, mkeys = mm_model()
  save_file({k: v.contiguous() for k, v in m.items()},
            os.path.join(HERE, "mm_model.safetensors"),
            metadata={"param_keys": ",".join(mkeys)})
  save_file(images(), os.path.join(HERE, "images.safetensors"))
  for f in sorted(os.listdir(HERE)):
    if f.endswith(".safetensors"):
      print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
  main()
