"""CPU oracle: a restatement of the reference `recurrentgemma/torch` path.

TEST INFRASTRUCTURE ONLY.  Nothing in the shipped package imports this
module; only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg use it, as the checker / CPU baseline.

Every function restates one reference function in eager PyTorch on the CPU,
keeping the reference's dtype and rounding points (bf16 storage, fp32 scan
state, fp32 softmax), and cites the lines it follows.  Parameters come in a
flat dict with the reference state-dict keys, so a state dict
from `cadence.Griffin` can be fed here unchanged.

Parity pinning: the environment refused execution of the
reference's Python, so this restatement is pinned by the reference tests'
known-answer vectors and invariants instead (RMSNorm KAT, attention-cache
update KAT, prefill-vs-sampler forward equivalence, scan dtype contract) --
see tests/test_oracle_kats.py.  Values the KATs do not cover are "parity
unpinned" against a live reference run.
"""

from __future__ import annotations

import math
from typing import Any

import torch
import torch.nn.functional as F

MIN_LOGIT = -2.3819763e38      # modules.py:29
MAX_WAVELENGTH = 10_000        # modules.py:30


# ---------------------------------------------------------------- layers.py

def rms_norm(x: torch.Tensor, scale: torch.Tensor, eps: float = 1e-6):
  """layers.py:70-78.  Every op rounds to x.dtype."""
  var = x.square().mean(dim=-1, keepdim=True)
  y = x * torch.rsqrt(var + eps)
  return y * (scale.view(*([1] * (x.ndim - 1)), -1) + 1)


def block_diagonal_linear(x, w, b):
  """layers.py:132-142: per-head  x[..,h,:] @ w[h] + b[h]."""
  h = w.shape[0]
  xs = x.unflatten(-1, (h, -1))
  y = torch.einsum("...hi,hij->...hj", xs, w) + b
  return y.flatten(-2)


def rnn_scan(x, a, reset, h0, acc_dtype=torch.float32):
  """layers.py:145-199.  fp32 state, separate mul and add per step."""
  assert x.ndim == 3 and a.shape == x.shape and a.dtype == x.dtype
  assert h0 is None or h0.dtype == acc_dtype
  a = a * ~reset[..., None]
  if x.shape[1] == 1:
    if h0 is None:
      return x, x[:, 0].to(acc_dtype)
    y = a.to(acc_dtype) * h0[:, None] + x.to(acc_dtype)
    return y.to(x.dtype), y[:, -1]
  h = torch.zeros(x[:, 0].shape, dtype=acc_dtype) if h0 is None else h0
  af, xf = a.to(acc_dtype), x.to(acc_dtype)
  y = torch.zeros_like(x)
  for t in range(x.shape[1]):
    h = af[:, t] * h + xf[:, t]
    y[:, t] = h.to(x.dtype)
  return y, h


def rg_lru(x, segment_pos, p: dict[str, torch.Tensor], prefix: str, h0=None):
  """layers.py:321-375 with the bf16 rounding chain of SURVEY App. A Q6."""
  reset = segment_pos == 0
  gate_x = torch.sigmoid(block_diagonal_linear(
      x, p[prefix + "input_gate.w"], p[prefix + "input_gate.b"]))
  gate_a = torch.sigmoid(block_diagonal_linear(
      x, p[prefix + "a_gate.w"], p[prefix + "a_gate.b"]))
  log_a = -8.0 * gate_a * F.softplus(p[prefix + "a_param"])
  a = torch.exp(log_a)
  a_sq = torch.exp(2 * log_a)
  gated_x = x * gate_x
  mult = torch.sqrt(1 - a_sq)
  mult = reset[..., None] + ~reset[..., None] * mult
  normalized = gated_x * mult.to(x.dtype)
  return rnn_scan(normalized, a, reset, h0)


def conv1d(x, segment_pos, w, b, cache=None, compat: bool = True):
  """layers.py:457-546 (+ the document mask of :592-633).

  compat=True keeps the reference mask, which only looks ahead over
  `range(1, shift - 1)` (Appendix A, Q3): for shift 3 the tap x[t-3] is
  dropped when pos[t-2] == 0; shifts 1 and 2 are never masked.
  compat=False applies the upstream mask (`range(1, shift + 1)`).
  """
  width = w.shape[0]
  out_len = x.shape[1]
  if cache is not None:
    assert out_len == 1 and cache.shape[1] == width - 1
    full = torch.cat([cache.to(x.dtype), x], dim=1)
    prompt = width - 1
    cache_dtype = cache.dtype
  else:
    full = x.clone()           # the reference masks views of x in place (Q4)
    prompt = 0
    cache_dtype = x.dtype
  notb = (segment_pos != 0)
  if notb.ndim == 1:
    notb = notb[None]
  acc = None
  for shift in range(min(width, prompt + out_len)):
    lo = max(prompt - shift, 0)
    hi = prompt + out_len - shift
    win = full[:, lo:hi]
    if cache is None:
      looks = range(1, shift - 1) if compat else range(1, shift + 1)
      m = torch.ones(win.shape[:2], dtype=torch.bool)
      for k in looks:
        m = m & notb[:, lo + k: hi + k]
      if compat:
        # layers.py:506,524: `x_window *= mask` on a view of x, so the
        # zeroed rows stay zero for the later shifts (no effect there: their
        # masks are supersets) and in the cache x[:, 1-width:] (:542) -- rows
        # L-7..L-4 of a width-8 cache when a document starts near the end
        full[:, lo:hi] *= m[..., None].to(x.dtype)
        win = full[:, lo:hi]
      else:
        win = win * m[..., None].to(x.dtype)
    if win.shape[1] < out_len:
      pad = torch.zeros(win.shape[0], out_len - win.shape[1], win.shape[2],
                        dtype=win.dtype)
      win = torch.cat([pad, win], dim=1)
    term = win * w[width - shift - 1][None, None]
    acc = term if acc is None else acc + term
  out = acc + b[None, None]
  new_cache = full[:, 1 - width:].to(cache_dtype)
  if new_cache.shape[1] < width - 1:
    pad = torch.zeros(new_cache.shape[0], width - 1 - new_cache.shape[1],
                      new_cache.shape[2], dtype=new_cache.dtype)
    new_cache = torch.cat([pad, new_cache], dim=1)
  return out, new_cache


def einsum_up(x, w, b):
  """layers.py:726-729 for eqn '...td,cdD->c...tD' (MLP up-projection)."""
  return torch.einsum("...td,cdD->c...tD", x, w) + b


def linear(x, weight, bias=None):
  return F.linear(x, weight, bias)


# --------------------------------------------------------------- modules.py

def rope_tables(positions: torch.Tensor, rope_dim: int, dtype):
  """sin/cos exactly as modules.py:73-81 computes them (fp32, then dtype)."""
  freq = torch.arange(rope_dim // 2)
  timescale = MAX_WAVELENGTH ** (2 * freq / rope_dim)
  inv = 1.0 / timescale
  ang = positions[..., None, None] * inv           # [b, t, 1, rope_dim/2]
  return torch.sin(ang).to(dtype), torch.cos(ang).to(dtype)


def apply_rope(x, positions):
  """modules.py:53-87: rotate the first half of the head dim."""
  half = x.shape[-1] // 2
  x_rope, x_pass = x[..., :half], x[..., half:]
  sin, cos = rope_tables(positions, half, x.dtype)
  a, b = x_rope[..., : half // 2], x_rope[..., half // 2:]
  return torch.cat([a * cos - b * sin, b * cos + a * sin, x_pass], dim=-1)


def causal_window_mask(qpos, kpos, window, qseg=None, kseg=None):
  """modules.py:90-127."""
  if qseg is not None:
    same = qseg[..., :, None] == kseg[..., None, :]
  else:
    same = (kpos >= 0)[..., None, :]
  causal = qpos[..., :, None] >= kpos[..., None, :]
  inwin = qpos[..., :, None] <= kpos[..., None, :] + window
  return same & causal & inwin


def prefill_mask(segment_pos, window):
  """modules.py:130-152: segment ids = cumsum(pos == 0), array positions."""
  seg = torch.cumsum(segment_pos == 0, dim=-1)
  idx = torch.arange(segment_pos.shape[-1])[None].expand_as(segment_pos)
  return causal_window_mask(idx, idx, window, seg, seg)


def cache_mask(seq_len, num_tokens, window):
  """modules.py:155-185: positions of the ring-buffer slots."""
  q = torch.arange(seq_len)[None] + num_tokens[:, None]
  k = num_tokens[:, None] // window
  idx = torch.arange(window)[None]
  now = idx + k * window
  prev = idx + (k - 1) * window
  kpos = torch.where(now < num_tokens[:, None], now, prev)
  kpos = torch.cat([kpos, q], dim=-1)
  return causal_window_mask(q, kpos, window)


def cache_from_prompt(keys, values, segment_pos, window):
  """modules.py:260-290 (roll by num_tokens, right-pad to the window)."""
  w = min(window, keys.shape[1])
  num_tokens = segment_pos[:, -1] + 1
  kk, vv = keys[:, -w:], values[:, -w:]
  rk = torch.empty_like(kk)
  rv = torch.empty_like(vv)
  for i in range(kk.shape[0]):
    s = int(num_tokens[i]) % window
    rk[i] = torch.roll(kk[i], shifts=s, dims=0)
    rv[i] = torch.roll(vv[i], shifts=s, dims=0)
  if w < window:
    pad = torch.zeros(kk.shape[0], window - w, *kk.shape[2:], dtype=kk.dtype)
    rk = torch.cat([rk, pad], dim=1)
    rv = torch.cat([rv, pad], dim=1)
  return dict(keys=rk, values=rv, num_tokens=num_tokens.to(torch.int32))


def local_attention(x, segment_pos, p, prefix, num_heads, window, cache=None,
                    return_cache=True):
  """modules.py:402-483 (MQA: one shared K/V head); the cache update runs
  only when return_cache (modules.py:445-451)."""
  b, t, d = x.shape
  hd = d // num_heads
  q = linear(x, p[prefix + "proj_q.weight"]).unflatten(-1, (num_heads, hd))
  k = linear(x, p[prefix + "proj_k.weight"]).unflatten(-1, (1, hd))
  v = linear(x, p[prefix + "proj_v.weight"]).unflatten(-1, (1, hd))
  q = apply_rope(q, segment_pos)
  k = apply_rope(k, segment_pos)
  if cache is not None:
    allk = torch.cat([cache["keys"], k], dim=1)
    allv = torch.cat([cache["values"], v], dim=1)
    mask = cache_mask(t, cache["num_tokens"], window)
    # modules.py:188-225 (_update_attention_cache): n_fill = min(window, t)
    n_fill = min(window, t)
    if not return_cache:
      new_cache = None
    elif n_fill == 1:
      # single-token decode writes the ring slot in place
      slot = cache["num_tokens"] % window
      nk, nv = cache["keys"].clone(), cache["values"].clone()
      for i in range(b):
        nk[i, int(slot[i])] = k[i, 0]
        nv[i, int(slot[i])] = v[i, 0]
      new_cache = dict(keys=nk, values=nv,
                       num_tokens=(cache["num_tokens"] + 1).to(torch.int32))
    elif n_fill == window:
      # prompt in chunks: a fresh cache from the new rows only
      new_cache = cache_from_prompt(k, v, segment_pos, window)
    else:
      raise NotImplementedError("modules.py:224-225")
  else:
    allk, allv = k, v
    mask = prefill_mask(segment_pos, window)
    new_cache = cache_from_prompt(k, v, segment_pos, window)
  logits = torch.einsum("btnh,bsnh->bnts", q, allk.expand(-1, -1, num_heads, -1))
  logits = logits * (hd ** -0.5)
  logits = torch.where(mask[:, None], logits, MIN_LOGIT).to(torch.float32)
  probs = torch.softmax(logits, dim=-1).to(x.dtype)
  enc = torch.einsum("bnts,bsnh->btnh", probs,
                     allv.expand(-1, -1, num_heads, -1))
  out = linear(enc.flatten(-2), p[prefix + "proj_final.weight"],
               p[prefix + "proj_final.bias"])
  return out, new_cache


def recurrent_block(x, segment_pos, p, prefix, cache=None, compat=True):
  """modules.py:612-660."""
  y = linear(x, p[prefix + "linear_y.weight"], p[prefix + "linear_y.bias"])
  xb = linear(x, p[prefix + "linear_x.weight"], p[prefix + "linear_x.bias"])
  xb, conv_state = conv1d(xb, segment_pos, p[prefix + "conv_1d.w"],
                          p[prefix + "conv_1d.b"],
                          None if cache is None else cache["conv1d_state"],
                          compat=compat)
  xb, h = rg_lru(xb, segment_pos, p, prefix + "rg_lru.",
                 None if cache is None else cache["rg_lru_state"])
  out = linear(xb * y, p[prefix + "linear_out.weight"],
               p[prefix + "linear_out.bias"])
  return out, dict(rg_lru_state=h, conv1d_state=conv_state)


def mlp_block(x, p, prefix):
  """modules.py:744-757 with tanh-GELU (modules.py:293-295)."""
  up = einsum_up(x, p[prefix + "ffw_up.w"], p[prefix + "ffw_up.b"])
  act = F.gelu(up[0], approximate="tanh") * up[1]
  return linear(act, p[prefix + "ffw_down.weight"], p[prefix + "ffw_down.bias"])


def residual_block(x, segment_pos, p, i, cfg, cache=None, compat=True):
  """modules.py:880-914."""
  pre = f"blocks.{i}."
  h = rms_norm(x, p[pre + "temporal_pre_norm.scale"])
  if cfg.block_types[i].name == "RECURRENT":
    h, new_cache = recurrent_block(h, segment_pos, p, pre + "recurrent_block.",
                                   cache, compat)
  else:
    h, new_cache = local_attention(h, segment_pos, p, pre + "attention_block.",
                                   cfg.num_heads, cfg.attention_window_size,
                                   cache)
  resid = h + x
  out = mlp_block(rms_norm(resid, p[pre + "channel_pre_norm.scale"]), p,
                  pre + "mlp_block.")
  return out + resid, new_cache


def embed(tokens, p, cfg):
  """modules.py:994-1001: gather, then * bf16(sqrt(width)) = 50.5 at 2560."""
  x = p["embedder.input_embedding"][tokens]
  if cfg.embeddings_scale_by_sqrt_dim:
    x = x * torch.tensor(math.sqrt(cfg.width)).to(torch.bfloat16)
  return x


def splice_positions(segment_pos, n_vis):
  """griffin.py:186-191 with n_vis generalised from 729 (App. A Q1/Q2)."""
  b = segment_pos.shape[0]
  head = torch.arange(n_vis, dtype=segment_pos.dtype)[None].expand(b, -1)
  return torch.cat([head, segment_pos], dim=-1)


def griffin_forward(p, cfg, tokens, segment_pos, cache=None, image_tokens=None,
                    return_logits=True, compat=True, last_only=False):
  """griffin.py:143-226 for a batch of independent rows.

  `image_tokens` [B, n_vis, width] (projector output, bf16) is spliced in
  front of the text exactly as griffin.py:179-191 does when the positions
  contain a 0 (the reference's `0 in segment_pos and img_path` test).
  """
  x = embed(tokens, p, cfg)
  if image_tokens is not None and bool((segment_pos == 0).any()):
    x = torch.cat([image_tokens.to(x.dtype), x], dim=1)
    segment_pos = splice_positions(segment_pos, image_tokens.shape[1])
  new_cache = {}
  for i in range(cfg.num_layers):
    name = f"blocks.{i}"
    x, new_cache[name] = residual_block(
        x, segment_pos, p, i, cfg, None if cache is None else cache[name],
        compat)
  if not return_logits:
    return None, new_cache
  if last_only:
    x = x[:, -1:]
  x = rms_norm(x, p["final_norm.scale"])
  logits = x @ p["embedder.input_embedding"].T
  c = cfg.logits_soft_cap
  if c:
    logits = torch.tanh(logits / c) * c
  return logits, new_cache


# ------------------------------------------------------ image preprocessing

def pil_resize_to_tensor(rgb_u8, size):
  """Resize((S, S), BICUBIC) + ToTensor exactly as the reference runs them
  (dino_siglip.py:12-16, 88-124, 148-151: torchvision on a PIL image calls
  `Image.resize(size, BICUBIC)`; ToTensor = permute + float / 255).  Pillow
  itself is the checker here: [H, W, 3] uint8 -> [3, S, S] fp32."""
  import numpy as np
  from PIL import Image
  img = Image.fromarray(np.ascontiguousarray(rgb_u8), "RGB")
  img = img.resize((size, size), Image.BICUBIC)
  return torch.from_numpy(np.array(img, dtype=np.uint8)).permute(
      2, 0, 1).contiguous().to(torch.float32).div(255)


def pil_resample_np(rgb_u8, size):
  """Restatement of Pillow's ImagingResample (libImaging/Resample.c,
  Pillow 12.x; third-party, not under /root/reference): precompute_coeffs
  (bicubic a = -0.5, support 2 * max(scale, 1)), normalize_coeffs_8bpc
  (22-bit fixed point), horizontal pass to uint8, then vertical pass.  The
  HIP kernel follows this; tests pin it against Pillow itself."""
  import numpy as np

  def cubic(x):
    a = -0.5
    x = abs(x)
    if x < 1.0:
      return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
      return (((x - 5) * x + 8) * x - 4) * a
    return 0.0

  def coeffs(in_size):
    scale = float(in_size) / size
    fs = max(scale, 1.0)
    support = 2.0 * fs
    ss = 1.0 / fs
    rows = []
    for i in range(size):
      center = (i + 0.5) * scale
      xmin = max(int(center - support + 0.5), 0)
      xmax = min(int(center + support + 0.5), in_size) - xmin
      w = [cubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
      ww = sum(w)
      w = [v / ww if ww != 0.0 else v for v in w]
      k = [int(-0.5 + v * (1 << 22)) if v < 0 else int(0.5 + v * (1 << 22))
           for v in w]
      rows.append((xmin, np.array(k, dtype=np.int64)))
    return rows

  def clip8(acc):
    return np.clip(acc >> 22, 0, 255).astype(np.uint8)

  src = np.asarray(rgb_u8, dtype=np.int64)
  h, w = src.shape[:2]
  tmp = np.empty((h, size, 3), dtype=np.uint8)
  for xx, (xmin, k) in enumerate(coeffs(w)):
    acc = (1 << 21) + np.tensordot(k, src[:, xmin:xmin + len(k)], axes=([0], [1]))
    tmp[:, xx] = clip8(acc)
  tmp = tmp.astype(np.int64)
  out = np.empty((size, size, 3), dtype=np.uint8)
  for yy, (ymin, k) in enumerate(coeffs(h)):
    acc = (1 << 21) + np.tensordot(k, tmp[ymin:ymin + len(k)], axes=([0], [0]))
    out[yy] = clip8(acc)
  return out


# ------------------------------------------------ vision tower + projector

def vit_features(pixels, p, prefix, vcfg, tower):
  """timm VisionTransformer.get_intermediate_layers(n={feature_block}).

  dino_siglip.py:65-86,148-156: fp32, per-encoder Normalize, patch-embed
  conv (k = s = 14, valid), pos-embed add then prefix concat
  (`no_embed_class`), `feature_block + 1` pre-LN blocks, no final norm,
  prefix tokens dropped.  timm itself is not vendored (unpinned).
  """
  f = torch.float32
  mean = torch.tensor(tower.mean, dtype=f).view(1, 3, 1, 1)
  std = torch.tensor(tower.std, dtype=f).view(1, 3, 1, 1)
  x = (pixels.to(f) - mean) / std
  x = F.conv2d(x, p[prefix + "patch_embed.proj.weight"].to(f),
               p[prefix + "patch_embed.proj.bias"].to(f),
               stride=tower.patch_size)
  x = x.flatten(2).transpose(1, 2)
  x = x + p[prefix + "pos_embed"].to(f)
  b = x.shape[0]
  pre = []
  if tower.class_token:
    pre.append(p[prefix + "cls_token"].to(f).expand(b, -1, -1))
  if tower.reg_tokens:
    pre.append(p[prefix + "reg_token"].to(f).expand(b, -1, -1))
  x = torch.cat(pre + [x], dim=1)
  h, hd = tower.num_heads, tower.head_dim
  for i in range(vcfg.blocks_run):
    bp = f"{prefix}blocks.{i}."
    g = lambda n: p[bp + n].to(f)
    y = F.layer_norm(x, (tower.width,), g("norm1.weight"), g("norm1.bias"), 1e-6)
    qkv = F.linear(y, g("attn.qkv.weight"), g("attn.qkv.bias"))
    qkv = qkv.unflatten(-1, (3, h, hd)).permute(2, 0, 3, 1, 4)
    att = torch.softmax((qkv[0] * hd ** -0.5) @ qkv[1].transpose(-1, -2), -1)
    y = (att @ qkv[2]).transpose(1, 2).flatten(2)
    y = F.linear(y, g("attn.proj.weight"), g("attn.proj.bias"))
    if tower.layer_scale:
      y = y * g("ls1.gamma")
    x = x + y
    y = F.layer_norm(x, (tower.width,), g("norm2.weight"), g("norm2.bias"), 1e-6)
    y = F.linear(y, g("mlp.fc1.weight"), g("mlp.fc1.bias"))
    y = F.gelu(y, approximate="tanh" if tower.gelu_tanh else "none")
    y = F.linear(y, g("mlp.fc2.weight"), g("mlp.fc2.bias"))
    if tower.layer_scale:
      y = y * g("ls2.gamma")
    x = x + y
  return x[:, tower.num_prefix_tokens:]


def vision_encoder(pixels, p, vcfg):
  """dino_siglip.py:133-156: cat(dino, siglip) along features -> fp32."""
  d = vit_features(pixels, p, "vis_encoder.dino.", vcfg, vcfg.dino)
  s = vit_features(pixels, p, "vis_encoder.siglip.", vcfg, vcfg.siglip)
  return torch.cat([d, s], dim=2)


def projector(feats, p):
  """projector/mlp.py:13-31: bf16 Linear-GELU(erf)-Linear-GELU-Linear."""
  x = feats.to(torch.bfloat16)
  idx = sorted({int(k.split(".")[2]) for k in p if k.startswith("projector.proj.")})
  for j, li in enumerate(idx):
    x = F.linear(x, p[f"projector.proj.{li}.weight"], p[f"projector.proj.{li}.bias"])
    if j < len(idx) - 1:
      x = F.gelu(x)
  return x


def image_tokens(pixels, p, vcfg):
  return projector(vision_encoder(pixels, p, vcfg), p)


# ---------------------------------------------------------------- sampler

def greedy_sample(p, cfg, prompt_tokens, steps, pixels=None, vcfg=None,
                  compat=True, lengths=None):
  """examples/cadence_sampler.py:185-298 + :112-182 (greedy, no EOS stop).

  Prompts are equal length (positions arange(T)) unless `lengths` gives
  left-padded lengths (pads at position -1).  Prefill runs
  tokens[:, :-1] (+ image), then one cached step on the last prompt token,
  then `steps - 1` decode steps.  Returns the generated tokens [B, steps]
  and the per-step logits [B, steps, V].
  """
  b, t = prompt_tokens.shape
  pos = torch.arange(t, dtype=torch.int32)[None].expand(b, -1).contiguous()
  if lengths is not None:   # left-padded prompts (cadence_sampler.py:198-201)
    pos = torch.clip(pos - t + lengths.to(torch.int32)[:, None], min=-1)
  img = image_tokens(pixels, p, vcfg) if pixels is not None else None
  if t > 1:
    _, cache = griffin_forward(p, cfg, prompt_tokens[:, :-1], pos[:, :-1],
                               image_tokens=img, return_logits=False,
                               compat=compat)
    logits, cache = griffin_forward(p, cfg, prompt_tokens[:, -1:], pos[:, -1:],
                                    cache=cache, compat=compat)
  else:
    logits, cache = griffin_forward(p, cfg, prompt_tokens, pos,
                                    image_tokens=img, compat=compat)
    logits = logits[:, -1:]
  out_tok = [logits[:, 0].argmax(-1)]
  out_logits = [logits[:, 0]]
  cur = pos[:, -1:] + 1
  for _ in range(steps - 1):
    logits, cache = griffin_forward(p, cfg, out_tok[-1][:, None].to(torch.int32),
                                    cur, cache=cache, compat=compat)
    out_tok.append(logits[:, 0].argmax(-1))
    out_logits.append(logits[:, 0])
    cur = cur + 1
  return torch.stack(out_tok, 1), torch.stack(out_logits, 1)
