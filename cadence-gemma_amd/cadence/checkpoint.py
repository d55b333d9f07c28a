"""Checkpoint loading and Flax <-> PyTorch parameter conversion (host side).

Reference:
  * `examples/cadence_sampler.py:436-448`: `torch.load(path)["params"]` ->
    `GriffinConfig.from_torch_params` -> `Griffin.load_state_dict(strict=False)`;
  * `recurrentgemma/conversion.py:48-127`: `flatten_nested_dict`,
    `flax_params_to_pytorch_state_dict`, `pytorch_state_dict_to_flax_params`
    (there through jax; here on numpy / torch arrays, since jax is not part of
    the MI355X stack: a Flax tree restored as numpy arrays converts the same
    way).

Files are read only with loaders that execute nothing from the file:
`torch.load(..., weights_only=True)` and safetensors.
"""

from __future__ import annotations

from typing import Any, Mapping

import numpy as np
import torch


def flatten_nested_dict(nested: Mapping[str, Any], prefix: str = "") -> dict[str, Any]:
  """conversion.py:48-62: {"a": {"b": x}} -> {"a.b": x}."""
  flat = {}
  for key, value in nested.items():
    name = prefix + key
    if isinstance(value, Mapping):
      flat.update(flatten_nested_dict(value, name + "."))
    else:
      flat[name] = value
  return flat


def _to_tensor(x, dtype: torch.dtype | None) -> torch.Tensor:
  t = x.detach().cpu() if isinstance(x, torch.Tensor) else torch.from_numpy(
      np.ascontiguousarray(np.asarray(x)))
  return t.to(dtype) if dtype is not None else t


def flax_params_to_state_dict(params: Mapping[str, Any],
                              dtype: torch.dtype | None = None
                              ) -> dict[str, torch.Tensor]:
  """conversion.py:65-83: Flax names -> torch names ("kernel" -> "weight"),
  2-D Linear kernels transposed ([in, out] -> [out, in]) except the Conv1D
  taps.  As in the reference, the flattened names keep whatever root the
  tree has: the whole {"params": ...} tree gives "params.blocks.0...." keys
  (strip them with `strip_params_prefix`), the subtree gives "blocks.0....".
  Arrays may be numpy (bf16 restored as float32 — pass dtype=torch.bfloat16)
  or torch tensors."""
  out = {}
  for key, value in flatten_nested_dict(params).items():
    key = key.replace("kernel", "weight")
    t = _to_tensor(value, dtype)
    if key.endswith("weight") and t.ndim == 2 and "conv1d" not in key:
      t = t.T.contiguous()
    out[key] = t
  return out


_TOP_LEVEL = ("blocks", "embedder", "final_norm", "vis_encoder", "projector")


def strip_params_prefix(state_dict: Mapping[str, Any]) -> dict[str, Any]:
  """Drops a leading "params." from every key (the reference's flattened
  whole-tree convention, conversion.py:100-104)."""
  return {(k[len("params."):] if k.startswith("params.") else k): v
          for k, v in state_dict.items()}


def state_dict_to_flax_params(state_dict: Mapping[str, torch.Tensor]
                              ) -> dict[str, Any]:
  """conversion.py:86-127: the inverse, as a {"params": {...}} tree of numpy
  arrays ("blocks.{i}" stays one level, as in the Flax module tree); bf16
  tensors come back as float32 numpy arrays (numpy has no bfloat16).  Keys
  may carry the reference's leading "params." (conversion.py:100-104
  asserts it) or not; any other root raises, as the reference's assert."""
  root: dict[str, Any] = {}
  for key, value in strip_params_prefix(state_dict).items():
    key = key.replace("weight", "kernel")
    t = value.detach().cpu()
    if t.dtype == torch.bfloat16:
      t = t.float()
    if key.endswith("kernel") and t.ndim == 2 and "conv1d" not in key:
      t = t.T
    path = key.split(".")
    if path[0] not in _TOP_LEVEL:
      raise ValueError(f"unexpected parameter {key!r}: the root must be one "
                       f"of {_TOP_LEVEL} (optionally under 'params.')")
    if path[0] == "blocks":
      path = [f"{path[0]}.{path[1]}"] + path[2:]
    node = root
    for p in path[:-1]:
      node = node.setdefault(p, {})
    node[path[-1]] = t.contiguous().numpy()
  return {"params": root}


def load_params(path: str, device=None, dtype: torch.dtype | None = None
                ) -> dict[str, torch.Tensor]:
  """Reads a torch state dict from `path` (.safetensors, or a torch file
  holding either the state dict or {"params": state dict} as the reference's
  checkpoints do) without executing anything from the file.  Keys come back
  without a leading "params."."""
  if path.endswith(".safetensors"):
    from safetensors.torch import load_file
    params = load_file(path)
  else:
    params = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(params, Mapping) and "params" in params and isinstance(
        params["params"], Mapping):
      params = params["params"]
    params = flatten_nested_dict(params) if any(
        isinstance(v, Mapping) for v in params.values()) else dict(params)
  out = {}
  for k, v in strip_params_prefix(params).items():
    if not isinstance(v, torch.Tensor):
      raise ValueError(f"{path}: entry {k!r} is not a tensor")
    out[k] = v.to(device=device, dtype=dtype if v.is_floating_point() else None)
  return out


def load_griffin(path: str, preset=None, device="cuda", dtype=torch.bfloat16,
                 vision=None, vision_params: str | Mapping | None = None,
                 **config_overrides):
  """The reference's load sequence (cadence_sampler.py:436-448) in one call:
  params -> `GriffinConfig.from_torch_params` -> `Griffin` ->
  `load_state_dict`.  Returns (model, config).

  The reference loads with strict=False, which would hide a misnamed key;
  here every parameter of the text model must come from the file, and keys
  the model does not have raise.  The reference gets its DINO / SigLIP
  weights from timm's pretrained download (dino_siglip.py:65-77), not from
  this file, so with `vision` set the tower + projector weights must be in
  the file or in `vision_params` (a path or a state dict with
  `vis_encoder.*` / `projector.*` keys); otherwise this raises rather than
  leave the tower at random init."""
  from . import common, griffin
  params = load_params(path)
  if vision_params is not None:
    extra = (load_params(vision_params) if isinstance(vision_params, str)
             else strip_params_prefix(vision_params))
    params = {**params, **extra}
  config = common.GriffinConfig.from_torch_params(
      {k: v for k, v in params.items()
       if not k.startswith(("vis_encoder.", "projector."))},
      preset=preset, **config_overrides)
  model = griffin.Griffin(config, device=device, dtype=dtype, vision=vision)
  res = model.load_state_dict({k: v.to(device) for k, v in params.items()},
                              strict=False)
  if res.unexpected_keys:
    raise ValueError(f"{path}: keys the model does not have: "
                     f"{sorted(res.unexpected_keys)[:8]}")
  if res.missing_keys:
    raise ValueError(
        f"{path}: parameters missing from the checkpoint: "
        f"{sorted(res.missing_keys)[:8]} ({len(res.missing_keys)} in all)"
        + ("; the vision tower and projector need `vision_params`"
           if any(k.startswith(("vis_encoder.", "projector."))
                  for k in res.missing_keys) else ""))
  return model, config
