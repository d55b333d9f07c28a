"""Checkpoint loading and Flax <-> torch conversion (CPU; one gpu test).

Reference: examples/cadence_sampler.py:436-448 (load sequence),
recurrentgemma/conversion.py:48-127 (conversion rules).
"""

import numpy as np
import pytest
import torch

import cadence
from cadence import checkpoint, common

RA = common.TemporalBlockType


def _cfg():
  return common.GriffinConfig(
      vocab_size=64, width=128, mlp_expanded_width=384, num_heads=2,
      block_types=(RA.RECURRENT, RA.ATTENTION), embeddings_scale_by_sqrt_dim=True,
      attention_window_size=32, logits_soft_cap=30.0)


def _state_dict():
  torch.manual_seed(0)
  m = cadence.Griffin(_cfg(), dtype=torch.bfloat16)
  g = torch.Generator().manual_seed(1)
  return {k: torch.randn(v.shape, generator=g).to(v.dtype)
          for k, v in m.state_dict().items()}


def test_flatten_nested_dict():
  assert checkpoint.flatten_nested_dict({"a": {"b": 1, "c": {"d": 2}}, "e": 3}) == {
      "a.b": 1, "a.c.d": 2, "e": 3}


def test_flax_round_trip_and_layout_rules():
  sd = _state_dict()
  flax = checkpoint.state_dict_to_flax_params(sd)
  p = flax["params"]
  # Flax tree: "blocks.{i}" one level, Linear kernels [in, out], conv taps kept
  lin = p["blocks.0"]["recurrent_block"]["linear_x"]["kernel"]
  assert lin.shape == tuple(sd["blocks.0.recurrent_block.linear_x.weight"].shape[::-1])
  conv = p["blocks.0"]["recurrent_block"]["conv_1d"]["w"]
  assert conv.shape == tuple(sd["blocks.0.recurrent_block.conv_1d.w"].shape)
  assert isinstance(lin, np.ndarray) and lin.dtype == np.float32
  # whole tree -> "params."-rooted names, as conversion.py:65-83 flattens it
  back = checkpoint.flax_params_to_state_dict(flax, dtype=torch.bfloat16)
  assert all(k.startswith("params.") for k in back)
  back = checkpoint.strip_params_prefix(back)
  assert set(back) == set(sd)
  assert set(checkpoint.flax_params_to_state_dict(p)) == set(sd)
  for k in sd:
    assert back[k].shape == sd[k].shape, k
    assert torch.equal(back[k], sd[k]), k


def test_reference_convention_keys():
  """pytorch_state_dict_to_flax_params (conversion.py:86-127) takes
  'params.'-prefixed keys and nests them under one 'params' root."""
  sd = _state_dict()
  ref_keys = {"params." + k: v for k, v in sd.items()}
  a = checkpoint.state_dict_to_flax_params(ref_keys)
  b = checkpoint.state_dict_to_flax_params(sd)
  assert set(a) == {"params"} and set(a["params"]) == set(b["params"])
  assert "params" not in a["params"]
  lin = "blocks.0"
  np.testing.assert_array_equal(
      a["params"][lin]["recurrent_block"]["linear_x"]["kernel"],
      b["params"][lin]["recurrent_block"]["linear_x"]["kernel"])
  with pytest.raises(ValueError):
    checkpoint.state_dict_to_flax_params({"params.bogus.w": torch.zeros(2)})


def test_load_params_weights_only_and_safetensors(tmp_path):
  sd = _state_dict()
  pt = tmp_path / "ckpt.pt"
  torch.save({"params": sd}, pt)          # the reference's checkpoint layout
  got = checkpoint.load_params(str(pt))
  assert set(got) == set(sd) and all(torch.equal(got[k], sd[k]) for k in sd)
  from safetensors.torch import save_file
  st = tmp_path / "ckpt.safetensors"
  save_file(sd, str(st))
  got = checkpoint.load_params(str(st), dtype=torch.float32)
  assert got["final_norm.scale"].dtype == torch.float32
  cfg = common.GriffinConfig.from_torch_params(
      got, embeddings_scale_by_sqrt_dim=True, attention_window_size=32,
      logits_soft_cap=30.0)
  assert cfg.block_types == _cfg().block_types and cfg.num_heads == 2


def test_load_griffin_strict_keys(tmp_path):
  """Missing / unexpected keys raise instead of leaving random weights
  (the reference loads with strict=False, cadence_sampler.py:448)."""
  sd = _state_dict()
  kw = dict(device="cpu", embeddings_scale_by_sqrt_dim=True,
            attention_window_size=32, logits_soft_cap=30.0)
  part = dict(sd)
  part.pop("blocks.1.mlp_block.ffw_down.bias")
  torch.save({"params": part}, tmp_path / "missing.pt")
  with pytest.raises(ValueError, match="missing"):
    cadence.load_griffin(str(tmp_path / "missing.pt"), **kw)
  extra = dict(sd)
  extra["blocks.0.recurrent_block.bogus"] = torch.zeros(3)
  torch.save({"params": extra}, tmp_path / "extra.pt")
  with pytest.raises(ValueError, match="does not have"):
    cadence.load_griffin(str(tmp_path / "extra.pt"), **kw)
  torch.save({"params": sd}, tmp_path / "text.pt")
  vis = common.VisionConfig(
      image_size=28,
      dino=common.ViTConfig("dino", 64, 1, 2, 128, class_token=True,
                            reg_tokens=4, layer_scale=True),
      siglip=common.ViTConfig("siglip", 64, 1, 2, 128),
      feature_block=0, projector_width=128)
  with pytest.raises(ValueError, match="vision_params"):
    cadence.load_griffin(str(tmp_path / "text.pt"), vision=vis, **kw)


def test_images_without_vision_tower_raise():
  m = cadence.Griffin(_cfg(), dtype=torch.bfloat16)
  tok = torch.zeros(1, 3, dtype=torch.int32)
  with pytest.raises(ValueError, match="vision"):
    m.embed_inputs(tok, torch.arange(3, dtype=torch.int32)[None],
                   images=torch.zeros(1, 3, 28, 28))


@pytest.mark.gpu
def test_load_griffin_matches_source_model(dev, tmp_path):
  cfg = _cfg()
  sd = {k: (v * 0.05 if v.ndim > 1 else v * 0.1) for k, v in _state_dict().items()}
  src = cadence.Griffin(cfg, device=dev, dtype=torch.bfloat16)
  src.load_state_dict({k: v.to(dev) for k, v in sd.items()})
  path = tmp_path / "ckpt.pt"
  torch.save({"params": sd}, path)
  model, cfg2 = cadence.load_griffin(str(path), device=dev,
                                     embeddings_scale_by_sqrt_dim=True,
                                     attention_window_size=32,
                                     logits_soft_cap=30.0)
  assert (cfg2.width, cfg2.block_types, cfg2.num_heads, cfg2.vocab_size) == (
      cfg.width, cfg.block_types, cfg.num_heads, cfg.vocab_size)
  tok = torch.randint(3, 64, (2, 9), dtype=torch.int32, device=dev)
  pos = torch.arange(9, dtype=torch.int32, device=dev)[None].repeat(2, 1)
  with torch.no_grad():
    a, _ = src(tok, pos)
    b, _ = model(tok, pos)
  assert torch.equal(a, b)
