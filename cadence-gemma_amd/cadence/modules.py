"""Griffin blocks on MI355X.

Public surface of the reference `recurrentgemma/torch/modules.py`: the cache
NamedTuples (:33-50), `LocalAttentionBlock` (:298-500), `RecurrentBlock`
(:503-685), `MLPBlock` (:688-757), `ResidualBlock` (:759-946) and `Embedder`
(:949-1006), with the same parameter names, initialisers, forward
signatures and cache-ownership rules (decode-mode attention caches are
updated in place and returned, modules.py:210-218).

Each block runs as a short chain of fused gfx950 kernels:
  recurrent:  rmsnorm -> [linear_y | linear_x] GEMM -> conv1d ->
              BDL-gates GEMM (gate chain fused) -> scan (x * y fused) ->
              linear_out GEMM (+bias +residual)
  attention:  rmsnorm -> [q | k | v] GEMM -> RoPE -> flash MQA ->
              proj_final GEMM (+bias +residual)
  MLP:        rmsnorm -> up GEMM (gelu_tanh(gate) * up fused) ->
              ffw_down GEMM (+bias +residual)
"""

from __future__ import annotations

import math
from typing import NamedTuple

import torch
from torch import nn

from . import common, layers, ops
from .layers import PackCache, _flat, positions_2d
from .tracing import trace


class RecurrentBlockCache(NamedTuple):
  rg_lru_state: torch.Tensor      # [B, E] fp32
  conv1d_state: torch.Tensor      # [B, W-1, E]


class AttentionBlockCache(NamedTuple):
  keys: torch.Tensor              # [B, window, 1, head_dim]
  values: torch.Tensor            # [B, window, 1, head_dim]
  num_tokens: torch.Tensor        # [B] int32


ResidualBlockCache = RecurrentBlockCache | AttentionBlockCache


def gelu(x: torch.Tensor) -> torch.Tensor:
  """tanh-approximated GELU (reference modules.py:293-295)."""
  return nn.functional.gelu(x, approximate="tanh")


def _out_proj(x2d, lin: nn.Linear, resid2d, norm, lazy=False):
  """Residual output projection, optionally fused with the RMSNorm that
  consumes it (returns (out, norm(out) or None)).  lazy: the consumer is a
  norm-aware decode GEMV, so decode rows come back unnormalised with the
  norm attached (ops.PackedRows.norm) and it applies the norm on load."""
  if norm is None:
    return ops.linear(x2d, lin.weight, lin.bias, resid=resid2d), None
  return ops.linear_rmsnorm(x2d, lin.weight, lin.bias, resid2d, norm, lazy=lazy)


class LocalAttentionBlock(nn.Module):
  """Local multi-query attention (one shared key/value head)."""

  def __init__(self, width: int, num_heads: int, window_size: int,
               final_w_init_variance_scale: float = 1.0, device=None,
               dtype=None):
    super().__init__()
    self.width = width
    self.num_heads = num_heads
    self.window_size = window_size
    self.final_w_init_variance_scale = final_w_init_variance_scale
    kw = dict(device=device, dtype=dtype)
    self.proj_q = nn.Linear(width, width, bias=False, **kw)
    self.proj_k = nn.Linear(width, self.head_dim, bias=False, **kw)
    self.proj_v = nn.Linear(width, self.head_dim, bias=False, **kw)
    self.proj_final = nn.Linear(width, width, bias=True, **kw)
    self._packed = PackCache()
    self._packed_rope = PackCache()
    self.reset_parameters()

  @property
  def head_dim(self) -> int:
    return self.width // self.num_heads

  def reset_parameters(self) -> None:
    for lin in (self.proj_q, self.proj_k, self.proj_v):
      self.w_init_(lin.weight)
    self.out_w_init_(self.proj_final.weight)
    nn.init.zeros_(self.proj_final.bias)

  def w_init_(self, w):
    nn.init.normal_(w, mean=0.0, std=math.sqrt(1.0 / self.width))

  def out_w_init_(self, w):
    nn.init.normal_(w, mean=0.0, std=math.sqrt(
        self.final_w_init_variance_scale / self.width))

  def qkv_weight(self):
    """[proj_q; proj_k; proj_v], zero rows appended up to a multiple of 64
    (the GEMM engines tile 64 columns; only narrow heads need them)."""
    def build():
      w = torch.cat([self.proj_q.weight, self.proj_k.weight, self.proj_v.weight])
      pad = (-w.shape[0]) % 64
      if pad:
        w = torch.cat([w, w.new_zeros(pad, w.shape[1])])
      return w.contiguous()
    return self._packed.get(
        [self.proj_q.weight, self.proj_k.weight, self.proj_v.weight], build)

  def qkv_weight_rope(self):
    """[proj_q; proj_k; proj_v] in cadence_qkv_rope_decode's row order."""
    return self._packed_rope.get(
        [self.proj_q.weight, self.proj_k.weight, self.proj_v.weight],
        lambda: self.qkv_weight()[:(self.num_heads + 2) * self.head_dim][ops.qkv_rope_permutation(
            self.num_heads, self.head_dim, self.proj_q.weight.device)].contiguous())

  def fused(self, xn2d, pos, b, t, cache, return_cache, resid2d, norm=None,
            lazy=False):
    """Attention branch on normalised rows; returns (resid + out,
    norm(resid + out) or None, cache)."""
    h, hd = self.num_heads, self.head_dim
    tuned = hd in (64, 128, 256)
    if cache is not None and t == 1 and b <= 32 and self.width <= 2560 and tuned:
      # decode: RoPE runs in the q|k|v projection's epilogue
      q, k, v = ops.qkv_rope_decode(xn2d, self.qkv_weight_rope(),
                                    pos.view(-1).to(torch.int32), h, hd)
    elif (tuned and isinstance(xn2d, torch.Tensor) and
          ops.qkv_rope_prefill_ok(b * t, h, hd, self.width)):
      # prompt pass: RoPE in the q|k|v GEMM's epilogue (one launch)
      q, k, v = ops.ops.qkv_rope_prefill(xn2d, self.qkv_weight_rope(),
                                         pos.view(-1).to(torch.int32), h, hd,
                                         ops.rope_table(xn2d.device, hd))
    else:
      qkv = ops.linear(xn2d, self.qkv_weight())[:, :(h + 2) * hd]
      q, k, v = ops.ops.rope_qkv(qkv, pos.view(-1), h, hd,
                                 ops.rope_table(qkv.device, hd) if tuned else None)
    if cache is None:
      # every attention block of a forward sees the same positions tensor:
      # its segment ids / starts are computed once and kept on it
      info = getattr(pos, "_cadence_segment_info", None)
      if info is None:
        info = ops.ops.segment_info(pos)
        pos._cadence_segment_info = info
      seg, start = info
      enc = ops.ops.local_attention(q, k, v, seg, start, b, t, h, hd,
                                    self.window_size)
      new_cache = None
      if return_cache:
        ck, cv, nt = ops.ops.kv_cache_fill(k, v, pos, self.window_size)
        new_cache = AttentionBlockCache(ck, cv, nt)
    else:
      n_fill = min(self.window_size, t)
      if return_cache and n_fill != 1 and n_fill != self.window_size:
        # reference modules.py:206-225 only updates a cache with 1 or
        # >= window tokens; it is called only when return_cache (:445-451)
        raise NotImplementedError()
      if t == 1 and tuned:
        enc = ops.local_attention_decode_(q, k, v, cache.keys, cache.values,
                                          cache.num_tokens, h)
        new_cache = cache if return_cache else None
      else:
        # a multi-token step against the cache (the prompt-in-chunks path,
        # n_fill == window) or a head dim the tuned decode kernel does not
        # cover: keys = [ring | new rows], mask from num_tokens
        enc = ops.ops.local_attention_cached(
            q, k, v, cache.keys, cache.values, cache.num_tokens, b, t, h, hd,
            self.window_size)
        new_cache = None
        if return_cache:
          if t == 1:      # in place, as the reference's n_fill == 1 branch
            ops.ops.kv_ring_update_(k, v, cache.keys, cache.values,
                                    cache.num_tokens, self.window_size)
            new_cache = cache
          else:           # _attention_cache_from_prompt of the new rows
            ck, cv, nt = ops.ops.kv_cache_fill(k, v, pos, self.window_size)
            new_cache = AttentionBlockCache(ck, cv, nt)
    out, hn = _out_proj(enc, self.proj_final, resid2d, norm, lazy)
    return out, hn, new_cache

  def forward(self, x: torch.Tensor, segment_pos: torch.Tensor,
              cache: AttentionBlockCache | None = None,
              return_cache: bool = True):
    b, t, d = x.shape
    pos = positions_2d(segment_pos, b, t)
    zero = torch.zeros(b * t, d, dtype=x.dtype, device=x.device)
    out, _, new_cache = self.fused(_flat(x), pos, b, t, cache, return_cache,
                                   zero)
    return out.view(b, t, d), new_cache

  @classmethod
  def init_cache(cls, batch_size: int, window_size: int, heads_dim: int,
                 dtype: torch.dtype, device=None) -> AttentionBlockCache:
    shape = (batch_size, window_size, 1, heads_dim)
    return AttentionBlockCache(
        keys=torch.zeros(shape, device=device, dtype=dtype),
        values=torch.zeros(shape, device=device, dtype=dtype),
        num_tokens=torch.zeros([batch_size], dtype=torch.int32, device=device))


class RecurrentBlock(nn.Module):
  """Conv1D + RG-LRU branch gated by a linear branch."""

  def __init__(self, width: int, num_heads: int, lru_width: int | None = None,
               conv1d_temporal_width: int = 4,
               final_w_init_variance_scale: float = 1.0, device=None,
               dtype=None, compat: bool = True):
    super().__init__()
    self.width = width
    self.num_heads = num_heads
    self.lru_width = lru_width or width
    self.conv1d_temporal_width = conv1d_temporal_width
    self.final_w_init_variance_scale = final_w_init_variance_scale
    kw = dict(device=device, dtype=dtype)
    self.linear_y = nn.Linear(width, self.lru_width, **kw)
    self.linear_x = nn.Linear(width, self.lru_width, **kw)
    self.linear_out = nn.Linear(self.lru_width, width, **kw)
    self.conv_1d = layers.Conv1D(self.lru_width, conv1d_temporal_width,
                                 compat=compat, **kw)
    self.rg_lru = layers.RGLRU(self.lru_width, num_heads, **kw)
    self._packed = PackCache()
    self.reset_parameters()

  def reset_parameters(self) -> None:
    self.w_init_(self.linear_x.weight)
    nn.init.zeros_(self.linear_x.bias)
    self.w_init_(self.linear_y.weight)
    nn.init.zeros_(self.linear_y.bias)
    self.out_w_init_(self.linear_out.weight)
    nn.init.zeros_(self.linear_out.bias)
    self.conv_1d.reset_parameters()
    self.rg_lru.reset_parameters()

  def w_init_(self, w):
    nn.init.normal_(w, mean=0.0, std=math.sqrt(1.0 / self.width))

  def out_w_init_(self, w):
    nn.init.normal_(w, mean=0.0, std=math.sqrt(
        self.final_w_init_variance_scale / self.lru_width))

  def yx_weight(self):
    src = [self.linear_y.weight, self.linear_x.weight, self.linear_y.bias,
           self.linear_x.bias]
    return self._packed.get(src, lambda: (
        torch.cat([self.linear_y.weight, self.linear_x.weight]).contiguous(),
        torch.cat([self.linear_y.bias, self.linear_x.bias]).contiguous()))

  def fused(self, xn2d, pos, b, t, cache, return_cache, resid2d,
            inplace_state: bool = False, norm=None, lazy=False):
    e = self.lru_width
    w, bias = self.yx_weight()
    if (inplace_state and return_cache and cache is not None and t == 1 and
        b <= 32 and cache.conv1d_state.is_contiguous() and
        cache.conv1d_state.dtype == xn2d.dtype):
      # decode: the y|x projection runs the x branch's Conv1D step in its
      # epilogue; conv / RG-LRU states are advanced in place by the kernels
      gated = ops.recurrent_decode_front_(
          xn2d, w, bias, self.conv_1d.w, self.conv_1d.b, cache.conv1d_state,
          self.rg_lru.packed(), pos.view(-1), cache.rg_lru_state)
      if gated is None:   # rows / shapes outside the one-launch plan
        yc = ops.linear_conv1d_(xn2d, w, bias, self.conv_1d.w, self.conv_1d.b,
                                cache.conv1d_state)     # [M, 2E]: y | conv(x)
        gated = self.rg_lru.step_(yc[:, e:], pos.view(-1), cache.rg_lru_state,
                                  yc[:, :e], packed_out=True)
      out, hn = _out_proj(gated, self.linear_out, resid2d, norm, lazy)
      return out, hn, cache
    yx = ops.linear(xn2d, w, bias)                       # [M, 2E]: y | x
    y_br, x_br = yx[:, :e], yx[:, e:]
    conv_out, conv_state = self.conv_1d.apply2d(
        x_br, pos, None if cache is None else cache.conv1d_state, b, t)
    h0 = None if cache is None else cache.rg_lru_state
    with trace("rg_lru"):
      gated, h_last = self.rg_lru.gates_scan(conv_out, pos.view(-1), h0, y_br, b, t)
    out, hn = _out_proj(gated, self.linear_out, resid2d, norm)
    if not return_cache:
      return out, hn, None
    if inplace_state and cache is not None:
      cache.rg_lru_state.copy_(h_last)
      cache.conv1d_state.copy_(conv_state)
      return out, hn, cache
    return out, hn, RecurrentBlockCache(rg_lru_state=h_last,
                                        conv1d_state=conv_state)

  def forward(self, x: torch.Tensor, segment_pos: torch.Tensor,
              cache: RecurrentBlockCache | None = None,
              return_cache: bool = True):
    b, t, d = x.shape
    pos = positions_2d(segment_pos, b, t)
    zero = torch.zeros(b * t, d, dtype=x.dtype, device=x.device)
    out, _, new_cache = self.fused(_flat(x), pos, b, t, cache, return_cache,
                                   zero)
    return out.view(b, t, d), new_cache

  @classmethod
  def init_cache(cls, batch_size: int, lru_width: int, dtype: torch.dtype,
                 conv1d_temporal_width: int = 4,
                 device=None) -> RecurrentBlockCache:
    return RecurrentBlockCache(
        rg_lru_state=layers.RGLRU.init_cache(batch_size, lru_width, device),
        conv1d_state=layers.Conv1D.init_cache(
            batch_size=batch_size, width=lru_width, dtype=dtype,
            conv1d_temporal_width=conv1d_temporal_width, device=device))


class MLPBlock(nn.Module):
  """Gated MLP: ffw_down(gelu_tanh(x W_gate + b) * (x W_up + b))."""

  def __init__(self, width: int, expanded_width: int,
               final_w_init_variance_scale: float = 1.0, device=None,
               dtype=None):
    super().__init__()
    self.width = width
    self.expanded_width = expanded_width
    self.final_w_init_variance_scale = final_w_init_variance_scale
    kw = dict(device=device, dtype=dtype)
    self.ffw_up = layers.Einsum((2, width, expanded_width),
                                (2, 1, 1, expanded_width),
                                "...td,cdD->c...tD", **kw)
    self.ffw_down = nn.Linear(expanded_width, width, **kw)
    self.reset_parameters()

  def reset_parameters(self) -> None:
    self.ffw_up.reset_parameters()
    nn.init.normal_(self.ffw_down.weight, mean=0.0, std=math.sqrt(
        self.final_w_init_variance_scale / self.expanded_width))
    nn.init.zeros_(self.ffw_down.bias)

  def fused(self, xn2d, resid2d, norm=None, lazy=False):
    """resid + MLP(xn); with `norm` also returns norm(that) (else None)."""
    w, bg, bu = self.ffw_up.gated_packed()
    act = ops.gated_gelu(xn2d, w, bg, bu)
    return _out_proj(act, self.ffw_down, resid2d, norm, lazy)

  def forward(self, x: torch.Tensor) -> torch.Tensor:
    zero = torch.zeros(_flat(x).shape, dtype=x.dtype, device=x.device)
    return self.fused(_flat(x), zero)[0].view(x.shape)


class ResidualBlock(nn.Module):
  """norm -> temporal block -> +res -> norm -> MLP -> +res."""

  def __init__(self, width: int, mlp_expanded_width: int, num_heads: int,
               attention_window_size: int,
               temporal_block_type: common.TemporalBlockType,
               lru_width: int | None = None, conv1d_temporal_width: int = 4,
               final_w_init_variance_scale: float = 1.0, device=None,
               dtype=None, compat: bool = True):
    super().__init__()
    self.width = width
    self.mlp_expanded_width = mlp_expanded_width
    self.num_heads = num_heads
    self.attention_window_size = attention_window_size
    self.temporal_block_type = temporal_block_type
    self.lru_width = lru_width
    self.conv1d_temporal_width = conv1d_temporal_width
    self.final_w_init_variance_scale = final_w_init_variance_scale
    kw = dict(device=device, dtype=dtype)
    self.temporal_pre_norm = layers.RMSNorm(width, **kw)
    if temporal_block_type == common.TemporalBlockType.RECURRENT:
      self.recurrent_block = RecurrentBlock(
          width, num_heads, lru_width, conv1d_temporal_width,
          final_w_init_variance_scale, compat=compat, **kw)
    else:
      self.attention_block = LocalAttentionBlock(
          width, num_heads, attention_window_size,
          final_w_init_variance_scale, **kw)
    self.channel_pre_norm = layers.RMSNorm(width, **kw)
    self.mlp_block = MLPBlock(width, mlp_expanded_width,
                              final_w_init_variance_scale, **kw)

  @property
  def temporal_block(self) -> nn.Module:
    if self.temporal_block_type == common.TemporalBlockType.RECURRENT:
      return self.recurrent_block
    return self.attention_block

  def reset_parameters(self) -> None:
    self.temporal_pre_norm.reset_parameters()
    self.temporal_block.reset_parameters()
    self.channel_pre_norm.reset_parameters()
    self.mlp_block.reset_parameters()

  def fused(self, x2d, pos, b, t, cache, return_cache,
            inplace_state: bool = False, xn=None, next_norm=None,
            next_lazy: bool = False):
    """One residual block on [B*T, D] rows.

    `xn` is temporal_pre_norm(x2d) when the previous block already produced
    it; `next_norm` is the RMSNorm that consumes this block's output (the
    next block's temporal_pre_norm or the final norm): each residual GEMM is
    fused with the norm that follows it.  Returns (out, next_norm(out) or
    None, cache).  next_lazy: `next_norm` is the next block's
    temporal_pre_norm, whose decode consumers (y|x + Conv1D, q|k|v + RoPE)
    apply it on load; channel_pre_norm always feeds the gated MLP GEMV, so
    it is left to that GEMV too."""
    if xn is None:
      xn = ops.rmsnorm(x2d, self.temporal_pre_norm.scale,
                       self.temporal_pre_norm.eps, packed=True)
    if self.temporal_block_type == common.TemporalBlockType.RECURRENT:
      resid, hn, new_cache = self.recurrent_block.fused(
          xn, pos, b, t, cache, return_cache, x2d, inplace_state,
          self.channel_pre_norm, lazy=True)
    else:
      resid, hn, new_cache = self.attention_block.fused(
          xn, pos, b, t, cache, return_cache, x2d, self.channel_pre_norm,
          lazy=True)
    out, out_norm = self.mlp_block.fused(hn, resid, next_norm, next_lazy)
    return out, out_norm, new_cache

  def forward(self, x: torch.Tensor, segment_pos: torch.Tensor,
              cache: ResidualBlockCache | None = None,
              return_cache: bool = True):
    b, t, d = x.shape
    pos = positions_2d(segment_pos, b, t)
    out, _, new_cache = self.fused(_flat(x), pos, b, t, cache, return_cache)
    return out.view(b, t, d), new_cache

  @classmethod
  def init_cache(cls, batch_size: int, width: int, num_heads: int,
                 attention_window_size: int,
                 temporal_block_type: common.TemporalBlockType,
                 dtype: torch.dtype, lru_width: int | None = None,
                 conv1d_temporal_width: int = 4,
                 device=None) -> ResidualBlockCache:
    if temporal_block_type == common.TemporalBlockType.RECURRENT:
      return RecurrentBlock.init_cache(batch_size, lru_width or width, dtype,
                                       conv1d_temporal_width, device)
    return LocalAttentionBlock.init_cache(batch_size, attention_window_size,
                                          width // num_heads, dtype, device)


class Embedder(nn.Module):
  """Token embedding; `decode` is the tied output projection."""

  def __init__(self, vocab_size: int, embed_dim: int, scale_by_sqrt_dim: bool,
               device=None, dtype=None):
    super().__init__()
    self.vocab_size = vocab_size
    self.embed_dim = embed_dim
    self.scale_by_sqrt_dim = scale_by_sqrt_dim
    self.input_embedding = nn.Parameter(torch.empty(
        [vocab_size, embed_dim], device=device, dtype=dtype))
    self.reset_parameters()

  def reset_parameters(self) -> None:
    nn.init.normal_(self.input_embedding, mean=0.0,
                    std=math.sqrt(1.0 / self.embed_dim))

  @property
  def scale(self) -> float:
    # the reference multiplies by a bf16 scalar: bf16(sqrt(2560)) = 50.5
    if not self.scale_by_sqrt_dim:
      return 1.0
    return float(torch.tensor(math.sqrt(self.embed_dim)).to(torch.bfloat16))

  def encode_into(self, tokens: torch.Tensor, out2d: torch.Tensor,
                  row_map=None):
    tok = tokens.reshape(-1).to(torch.int32).contiguous()
    m = tok.numel()
    div, mul, off = row_map if row_map is not None else (max(m, 1), 0, 0)
    ops.ops.embed_(tok, self.input_embedding, self.scale, out2d, div, mul, off)

  def encode_packed(self, tokens: torch.Tensor, norm):
    """The decode step's input rows (M <= 32): (x [M, D] row-major, the same
    rows as PackedRows carrying `norm`, the first block's temporal_pre_norm,
    which its decode GEMVs apply on load)."""
    tok = tokens.reshape(-1).to(torch.int32).contiguous()
    m, d = tok.numel(), self.embed_dim
    x = torch.empty(m, d, dtype=self.input_embedding.dtype, device=tok.device)
    xp = ops.packed_empty(m, d, tok.device)
    ops.ops.embed_packed_(tok, self.input_embedding, self.scale, x, xp)
    return x, ops.PackedRows(xp, m, d, norm, x)

  def encode_packed_into(self, tokens: torch.Tensor, x: torch.Tensor, xp: torch.Tensor):
    """encode_packed into given buffers (a captured decode loop's rows)."""
    tok = tokens.reshape(-1).to(torch.int32).contiguous()
    ops.ops.embed_packed_(tok, self.input_embedding, self.scale, x, xp)

  def encode(self, x: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.numel(), self.embed_dim, dtype=self.input_embedding.dtype,
                      device=x.device)
    self.encode_into(x, out)
    return out.view(*x.shape, self.embed_dim)

  def decode(self, x: torch.Tensor) -> torch.Tensor:
    logits = ops.gemm_logits(_flat(x), self.input_embedding, 0.0)
    return logits.view(*x.shape[:-1], self.vocab_size)
