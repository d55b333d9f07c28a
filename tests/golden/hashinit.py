"""Device-independent synthetic weights and inputs for the full-size fixtures.

TEST INFRASTRUCTURE.  The full-size golden fixtures (make_golden_full.py)
need the 2B Griffin + the two 23-block towers (3.4 G parameters) on both
sides: on this container's CPU, where the oracle produces the expected
vectors, and on the GPU box, where the HIP path is checked.  torch's own
random init is not reproducible across devices and takes ~2 minutes on
the CPU, so the fixture weights come from an integer hash instead:

  value(i) = (lowbias32(i ^ seed) >> 8) / 2^24 - 0.5   (exact in fp32)
             * (std * sqrt(12))                          (one fp32 multiply)
             -> bf16                                     (round to nearest even)

Every step is exact integer arithmetic or a single correctly rounded IEEE
operation, so CPU and GPU produce bit-identical tensors (uniform noise with
the requested standard deviation).  The few parameters that need
transcendentals (the RG-LRU `a_param`, rnn_param_init of
recurrentgemma/torch/layers.py:202-221) are small and always computed on
the CPU.  The std per tensor follows the reference init recipes by name
(layers.py:66-68,122-130,291-299; modules.py:361-380,572-590,733-742,
986-992; timm ViT: 0.02), with norms, biases and LayerScale perturbed away
from their identity init so every path carries signal.
"""

from __future__ import annotations

import math

import torch

_M32 = 0xFFFFFFFF
_CHUNK = 1 << 25


def _mul32(x: torch.Tensor, m: int) -> torch.Tensor:
  """(x * m) mod 2^32 for int64 x in [0, 2^32) without int64 overflow."""
  lo = x * (m & 0xFFFF)
  hi = ((x * (m >> 16)) & 0xFFFF) << 16
  return (lo + hi) & _M32


def _lowbias32(x: torch.Tensor) -> torch.Tensor:
  x = x ^ (x >> 16)
  x = _mul32(x, 0x7FEB352D)
  x = x ^ (x >> 15)
  x = _mul32(x, 0x846CA68B)
  return x ^ (x >> 16)


def hash_uniform(n: int, seed: int, device, offset: int = 0) -> torch.Tensor:
  """n fp32 values k / 2^24 in [0, 1), exact, identical on every device."""
  out = torch.empty(n, dtype=torch.float32, device=device)
  s = (seed * 0x9E3779B1) & _M32
  for lo in range(0, n, _CHUNK):
    hi = min(n, lo + _CHUNK)
    i = torch.arange(lo + offset, hi + offset, dtype=torch.int64, device=device)
    h = _lowbias32((i & _M32) ^ s ^ ((i >> 32) * 0x85EBCA6B & _M32))
    out[lo:hi] = (h >> 8).to(torch.float32) * (2.0 ** -24)
  return out


def hash_tensor(shape, seed: int, std: float, mean: float = 0.0, device="cpu",
                dtype=torch.bfloat16) -> torch.Tensor:
  n = math.prod(shape)
  u = hash_uniform(n, seed, device) - 0.5          # exact
  v = u * torch.tensor(std * math.sqrt(12.0), dtype=torch.float32)
  if mean:
    v = v + torch.tensor(mean, dtype=torch.float32)
  return v.to(dtype).view(*shape)


def _rnn_a_param(n: int, seed: int) -> torch.Tensor:
  """rnn_param_init(min_rad=0.9, max_rad=0.999) (layers.py:202-221) on
  hashed uniforms, on the CPU in float64."""
  u = hash_uniform(n, seed, "cpu").double()
  lo, hi = 0.9 ** 2 + 1e-8, 0.999 ** 2 + 1e-8
  a = 0.5 * torch.log(lo + u * (hi - lo))
  return torch.log(torch.exp(-a) - 1.0)


def param_spec(name: str, shape, num_layers: int = 0):
  """(kind, std, mean) for one state-dict entry."""
  if name.startswith("vis_encoder."):
    if name.endswith(("norm1.weight", "norm2.weight")):
      return "u", 0.1, 1.0
    if name.endswith(("ls1.gamma", "ls2.gamma")):
      return "u", 0.05, 0.2
    if name.endswith("patch_embed.proj.weight"):
      return "u", 1.0 / math.sqrt(math.prod(shape[1:])), 0.0
    if name.endswith(".bias"):
      return "u", 0.02, 0.0
    return "u", 0.02, 0.0          # Linear weights, pos_embed, cls/reg tokens
  if name.startswith("projector."):
    if name.endswith(".bias"):
      return "u", 0.02, 0.0
    return "u", 1.0 / math.sqrt(shape[-1]), 0.0
  if name.endswith("rg_lru.a_param"):
    return "a", 0.0, 0.0
  if name.endswith(".scale"):                        # RMSNorm (scale + 1)
    return "u", 0.1, 0.0
  if name.endswith((".bias", ".b")):
    return "u", 0.05, 0.0
  if name == "embedder.input_embedding":
    # 1.5x the reference's 1/sqrt(D): logits of a few logits' spread, so
    # greedy top-1 / top-2 margins fall mostly in 0.3-3
    return "u", 1.5 / math.sqrt(shape[-1]), 0.0
  if name.endswith("conv_1d.w"):
    return "u", math.sqrt(0.01 * 4 / shape[0]), 0.0  # temporal taps
  # residual-writing projections at 5 / sqrt(fan_in) (the reference scales
  # them by sqrt(2 / num_layers)): with the tied embedding, the input token's
  # own embedding (x 50.5) stays in the residual stream, and at 1 / sqrt(fan_in)
  # it still dominated the last position (greedy repeated the last prompt
  # token with a 6-9 logit margin, consecutive steps' logits 0.97 cosine).
  # At 5x the blocks carry the logits: greedy continuations vary and the
  # decode steps see changing inputs.
  if name.endswith(("linear_out.weight", "proj_final.weight", "ffw_down.weight")):
    return "u", 5.0 / math.sqrt(shape[-1]), 0.0
  if name.endswith("ffw_up.w"):                      # [2, D, F]
    return "u", 1.0 / math.sqrt(shape[-2]), 0.0
  if name.endswith(("input_gate.w", "a_gate.w")):    # [H, bw, bw]
    return "u", 1.0 / math.sqrt(shape[-2]), 0.0
  return "u", 1.0 / math.sqrt(shape[-1]), 0.0         # nn.Linear [out, in]


def hash_params(shapes: dict, seed: int, num_layers: int, device="cpu",
                dtype=torch.bfloat16) -> dict:
  """name -> tensor for every (name, shape) of a state dict, sorted by name
  so each tensor's hash seed is stable."""
  out = {}
  for j, name in enumerate(sorted(shapes)):
    shape = tuple(shapes[name])
    kind, std, mean = param_spec(name, shape, num_layers)
    pseed = seed * 100003 + j
    if kind == "a":
      out[name] = _rnn_a_param(math.prod(shape), pseed).to(dtype).view(
          *shape).to(device)
    else:
      out[name] = hash_tensor(shape, pseed, std, mean, device, dtype)
  return out


def hash_pixels(b: int, size: int, seed: int, device="cpu") -> torch.Tensor:
  """[B, 3, S, S] fp32 in [0, 1), like torch.rand images."""
  return hash_uniform(b * 3 * size * size, seed, device).view(b, 3, size, size)


def hash_tokens(b: int, t: int, vocab: int, seed: int, bos: int = 2) -> torch.Tensor:
  """[B, T] int32 in [3, vocab) with BOS first (bench.py's prompt layout)."""
  u = hash_uniform(b * t, seed, "cpu").double()
  tok = (3 + torch.floor(u * (vocab - 3))).to(torch.int32).view(b, t)
  tok[:, 0] = bos
  return tok


def checksums(p: dict) -> torch.Tensor:
  """float64 sum per tensor (sorted names); on the GPU compare with a
  relative tolerance (the reduction order differs)."""
  return torch.tensor([p[k].sum(dtype=torch.float64).item() for k in sorted(p)],
                      dtype=torch.float64)


def probes(p: dict, n: int = 16) -> torch.Tensor:
  """n values at fixed strided offsets of every tensor, as fp32: compared
  bit-exactly, they prove the device rebuild is the fixture's weights."""
  rows = []
  for k in sorted(p):
    flat = p[k].reshape(-1)
    idx = (torch.arange(n, dtype=torch.int64) * (flat.numel() - 1) // (n - 1)).to(
        flat.device)
    rows.append(flat[idx].float().cpu())
  return torch.stack(rows)
