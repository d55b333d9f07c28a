"""Base layers of the Griffin stack on MI355X.

Same public surface as the reference `recurrentgemma/torch/layers.py`
(`RMSNorm` :35-78, `BlockDiagonalLinear` :81-142, `rnn_scan` :145-199,
`rnn_param_init` :202-221, `RGLRU` :241-386, `Conv1D` :389-676, `Einsum`
:679-729): constructor arguments, parameter names/shapes (state-dict keys),
initialisers and `forward` signatures are kept.  The arithmetic runs in the
gfx950 kernels behind `torch.ops.cadence` (see ops.py); tensors must live on
the GPU.  Packed weight layouts for the fused kernels are derived lazily and
re-derived whenever a parameter is modified (load_state_dict, in-place init).
"""

from __future__ import annotations

import math
from typing import Callable, Sequence

import torch
import torch.nn.functional as F
from torch import nn

from . import ops


class PackCache:
  """Caches a derived (packed) weight until its source parameters change."""

  def __init__(self):
    self._sig = None
    self._val = None

  def get(self, sources: Sequence[torch.Tensor], build: Callable[[], object]):
    sig = tuple((t.data_ptr(), t._version, t.device) for t in sources)
    if sig != self._sig:
      with torch.no_grad():
        self._val = build()
      self._sig = sig
    return self._val


def _flat(x: torch.Tensor) -> torch.Tensor:
  return x.reshape(-1, x.shape[-1])


def positions_2d(segment_pos: torch.Tensor, b: int, t: int) -> torch.Tensor:
  """The reference auto-unsqueezes 1-D positions (layers.py:342-343)."""
  if segment_pos.shape != (b, t):
    segment_pos = segment_pos[None, :]
  assert segment_pos.shape == (b, t), segment_pos.shape
  if segment_pos.dtype != torch.int32:
    segment_pos = segment_pos.to(torch.int32)
  return segment_pos.contiguous()


class RMSNorm(nn.Module):
  """RMSNorm with a zero-initialised `scale` used as (scale + 1)."""

  def __init__(self, width: int, eps: float = 1e-6, device=None, dtype=None):
    super().__init__()
    self.width = width
    self.eps = eps
    self.scale = nn.Parameter(torch.empty([width], device=device, dtype=dtype))
    self.reset_parameters()

  def reset_parameters(self) -> None:
    nn.init.zeros_(self.scale)

  def forward(self, x: torch.Tensor) -> torch.Tensor:
    return ops.rmsnorm(_flat(x), self.scale, self.eps).view(x.shape)


class BlockDiagonalLinear(nn.Module):
  """`num_blocks` independent [block, block] linears over slices of x."""

  def __init__(self, width: int, num_blocks: int,
               w_init_variance_scale: float = 1.0, device=None, dtype=None):
    super().__init__()
    self.width = width
    self.num_blocks = num_blocks
    self.w_init_variance_scale = w_init_variance_scale
    self.block_width = width // num_blocks
    bw = self.block_width
    self.w = nn.Parameter(torch.empty([num_blocks, bw, bw], device=device,
                                      dtype=dtype))
    self.b = nn.Parameter(torch.empty([num_blocks, bw], device=device,
                                      dtype=dtype))
    self._packed = PackCache()
    self.reset_parameters()

  def reset_parameters(self) -> None:
    self.w_init_(self.w)
    nn.init.zeros_(self.b)

  def w_init_(self, w: torch.Tensor) -> None:
    nn.init.normal_(w, mean=0.0,
                    std=math.sqrt(self.w_init_variance_scale / self.block_width))

  def _weights_nk(self):
    # per block [out, in] (nn.Linear layout)
    return self._packed.get([self.w], lambda: self.w.transpose(1, 2).contiguous())

  def forward(self, x: torch.Tensor) -> torch.Tensor:
    wt = self._weights_nk()
    x2 = _flat(x)
    out = torch.empty_like(x2)
    bw = self.block_width
    for h in range(self.num_blocks):
      ops.linear(x2[:, h * bw:(h + 1) * bw], wt[h], self.b[h],
                 out=out[:, h * bw:(h + 1) * bw])
    return out.view(x.shape)


def rnn_scan(x: torch.Tensor, a: torch.Tensor, reset: torch.Tensor,
             h0: torch.Tensor | None, acc_dtype: torch.dtype = torch.float32):
  """Linear recurrence h_t = a_t * h_{t-1} + x_t (reference layers.py:145-199).

  x, a: [B, T, E] bf16; reset: [B, T] bool; h0: [B, E] fp32 or None.
  Returns (y [B, T, E] in x.dtype, h_last [B, E] fp32).
  """
  assert x.ndim == 3
  assert a.shape == x.shape[-a.ndim:]
  assert a.dtype == x.dtype
  assert h0 is None or h0.dtype == acc_dtype
  if acc_dtype != torch.float32:
    raise NotImplementedError("the MI355X scan accumulates in fp32")
  b, t, e = x.shape
  pos_like = (~reset).to(torch.int32).contiguous()   # 0 where reset
  y, h = ops.ops.rnn_scan(_flat(x), _flat(a), pos_like,
                          None if h0 is None else h0.contiguous(), None, b, t)
  return y.view(b, t, e), h


def rnn_param_init(tensor: torch.Tensor, min_rad: float, max_rad: float,
                   transform: str = "softplus", eps: float = 1e-8):
  """A = exp(-softplus(param)) uniform on the ring [min_rad, max_rad]."""
  if transform != "softplus":
    raise NotImplementedError()
  with torch.no_grad():
    tensor.uniform_(min_rad ** 2 + eps, max_rad ** 2 + eps)
    tensor.log_().mul_(0.5)                 # log |A|
    return tensor.neg_().exp_().sub_(1.0).log_()   # softplus^-1(-log |A|)


def _block_diag_groups(w: torch.Tensor, g: int) -> torch.Tensor:
  """[H, bw, bw] -> [H / g, g bw, g bw]: each group of g blocks on the
  diagonal of one zero matrix."""
  if g == 1:
    return w
  h, bw, _ = w.shape
  out = torch.zeros(h // g, g * bw, g * bw, dtype=w.dtype, device=w.device)
  for i in range(g):
    out[:, i * bw:(i + 1) * bw, i * bw:(i + 1) * bw] = w.view(h // g, g, bw, bw)[:, i]
  return out


class RGLRU(nn.Module):
  """Real-Gated Linear Recurrent Unit."""

  def __init__(self, width: int, num_heads: int,
               w_init_variance_scale: float = 1.0, device=None, dtype=None):
    super().__init__()
    self.width = width
    self.num_heads = num_heads
    self.w_init_variance_scale = w_init_variance_scale
    self.a_param = nn.Parameter(torch.empty([width], device=device, dtype=dtype))
    self.input_gate = BlockDiagonalLinear(width, num_heads,
                                          w_init_variance_scale, device, dtype)
    self.a_gate = BlockDiagonalLinear(width, num_heads, w_init_variance_scale,
                                      device, dtype)
    self._packed = PackCache()
    self.reset_parameters()

  def reset_parameters(self) -> None:
    self.input_gate.reset_parameters()
    self.a_gate.reset_parameters()
    self.a_param_init(self.a_param)

  def a_param_init(self, w: torch.Tensor) -> torch.Tensor:
    return rnn_param_init(w, min_rad=0.9, max_rad=0.999)

  def gate_blocks(self) -> int:
    """Heads merged into one block of the gate GEMM.  The grouped GEMM tiles
    64 columns per block; narrower heads (the reference grid's width 128 x
    16 heads: 8 wide) are merged G at a time into block-diagonal super-blocks
    whose off-diagonal weights are zero -- the sums are the same (a zero
    product adds exactly 0), so nothing is approximated."""
    h, bw = self.num_heads, self.width // self.num_heads
    for g in range(1, h + 1):
      if h % g == 0 and (g * bw) % 64 == 0:
        return g
    raise NotImplementedError(
        f"RG-LRU width {self.width} with {h} heads: no head grouping gives a "
        "block width that is a multiple of 64")

  def packed(self):
    """(W [H', 2*bw', bw'] interleaved per 32 rows, bias_x, bias_a,
    softplus(a)); H' = H / G super-blocks of bw' = G * bw (gate_blocks)."""
    def build():
      g = self.gate_blocks()
      h, bw = self.num_heads // g, g * (self.width // self.num_heads)
      wx = _block_diag_groups(self.input_gate.w, g).transpose(1, 2)   # [H', out, in]
      wa = _block_diag_groups(self.a_gate.w, g).transpose(1, 2)
      w = torch.stack([wx.reshape(h, bw // 32, 32, bw),
                       wa.reshape(h, bw // 32, 32, bw)], dim=2)
      w = w.reshape(h, 2 * bw, bw).contiguous()
      sp = F.softplus(self.a_param)                   # bf16, rounded once
      return (w, self.input_gate.b.reshape(-1).contiguous(),
              self.a_gate.b.reshape(-1).contiguous(), sp.contiguous())
    return self._packed.get([self.input_gate.w, self.a_gate.w, self.a_param,
                             self.input_gate.b, self.a_gate.b], build)

  def gates(self, x2d: torch.Tensor, pos_flat: torch.Tensor):
    """Fused BDL x2 + gate chain -> (a with resets zeroed, normalized x)."""
    w, bx, ba, sp = self.packed()
    return ops.rglru_gates(x2d, w, bx, ba, sp, pos_flat)

  def gates_scan(self, x2d: torch.Tensor, pos_flat: torch.Tensor, h0, gate,
                 b: int, t: int):
    """Prefill: gates then rnn_scan (a with resets zeroed, so no positions)
    joined with `gate` -> (bf16(h) [* gate] [B*T, E], h_last [B, E]); one
    fused launch where the kernel's plan takes the shape (enough sequences x
    blocks to fill the chip), the two kernels otherwise."""
    w, bx, ba, sp = self.packed()
    h, two_bw, bw = w.shape
    if ops.rglru_scan_plan(x2d, gate, b, t, h, bw):
      return ops.ops.rglru_scan(x2d, w, bx, ba, sp, pos_flat, h0, gate, b, t)
    a, nx = ops.rglru_gates(x2d, w, bx, ba, sp, pos_flat)
    return ops.ops.rnn_scan(nx, a, None, h0, gate, b, t)

  def step_(self, x2d: torch.Tensor, pos_flat: torch.Tensor, h: torch.Tensor,
            gate: torch.Tensor | None = None, packed_out: bool = False):
    """One token per row (T = 1): gates + scan step fused, `h` updated in
    place; returns bf16(h) [* gate] (PackedRows when `packed_out` and the
    rows qualify: the decode path's linear_out consumes it)."""
    w, bx, ba, sp = self.packed()
    return ops.rglru_step_(x2d, w, bx, ba, sp, pos_flat, h, gate,
                           None if packed_out else False)

  def forward(self, x: torch.Tensor, segment_pos: torch.Tensor,
              cache: torch.Tensor | None = None, return_cache: bool = True):
    b, t, e = x.shape
    pos = positions_2d(segment_pos, b, t)
    a, nx = self.gates(_flat(x), pos.view(-1))
    y, h = ops.ops.rnn_scan(nx, a, None, None if cache is None else cache,
                            None, b, t)
    return y.view(b, t, e), (h if return_cache else None)

  @classmethod
  def init_cache(cls, batch_size: int, width: int, device=None) -> torch.Tensor:
    return torch.zeros((batch_size, width), dtype=torch.float32, device=device)


class Conv1D(nn.Module):
  """Causal depthwise temporal convolution with a document mask.

  `compat=True` (default) reproduces the reference mask exactly, including
  its look-ahead off-by-two (layers.py:629).
  """

  def __init__(self, width: int, temporal_width: int,
               w_init_variance_scale: float = 0.01, device=None, dtype=None,
               compat: bool = True):
    super().__init__()
    self.width = width
    self.temporal_width = temporal_width
    self.w_init_variance_scale = w_init_variance_scale
    self.compat = compat
    self.w = nn.Parameter(torch.empty([temporal_width, width], device=device,
                                      dtype=dtype))
    self.b = nn.Parameter(torch.empty([width], device=device, dtype=dtype))
    self.reset_parameters()

  def reset_parameters(self) -> None:
    self.w_init_(self.w)
    nn.init.zeros_(self.b)

  def w_init_(self, w: torch.Tensor) -> None:
    nn.init.normal_(w, mean=0.0, std=math.sqrt(self.w_init_variance_scale /
                                               self.temporal_width))

  def apply2d(self, x2d, pos, cache, b, t):
    return ops.ops.conv1d(x2d, self.w, self.b, pos, cache, b, t, self.compat)

  def forward(self, x: torch.Tensor, segment_pos: torch.Tensor,
              cache: torch.Tensor | None = None, return_cache: bool = True):
    b, t, e = x.shape
    pos = positions_2d(segment_pos, b, t) if cache is None else \
        torch.ones(b, t, dtype=torch.int32, device=x.device)
    out, new_cache = self.apply2d(_flat(x), pos, cache, b, t)
    return out.view(b, t, e), (new_cache if return_cache else None)

  @classmethod
  def init_cache(cls, *, batch_size: int, width: int, dtype: torch.dtype,
                 conv1d_temporal_width: int = 4, device=None) -> torch.Tensor:
    return torch.zeros((batch_size, conv1d_temporal_width - 1, width),
                       dtype=dtype, device=device)


class Einsum(nn.Module):
  """Parameterised einsum; the MI355X path implements the MLP up-projection
  equation '...td,cdD->c...tD' (the only one the reference uses)."""

  def __init__(self, w_shape: Sequence[int], b_shape: Sequence[int], eqn: str,
               w_init_variance_scale: float = 1.0, device=None, dtype=None):
    super().__init__()
    self.w_shape = tuple(w_shape)
    self.b_shape = tuple(b_shape)
    self.eqn = eqn
    self.w_init_variance_scale = w_init_variance_scale
    self.w = nn.Parameter(torch.empty(self.w_shape, device=device, dtype=dtype))
    self.b = nn.Parameter(torch.empty(self.b_shape, device=device, dtype=dtype))
    self._packed = PackCache()
    self.reset_parameters()

  def reset_parameters(self) -> None:
    self.w_init_(self.w)
    nn.init.zeros_(self.b)

  def w_init_(self, w: torch.Tensor) -> None:
    nn.init.normal_(w, mean=0.0,
                    std=math.sqrt(self.w_init_variance_scale / self.w_shape[1]))

  def _check_eqn(self):
    if self.eqn.replace(" ", "") != "...td,cdD->c...tD":
      raise NotImplementedError(f"einsum {self.eqn!r} has no MI355X kernel")

  def weights_nk(self):
    """[c, D_out, d_in] copies of w (nn.Linear layout)."""
    return self._packed.get([self.w], lambda: self.w.transpose(1, 2).contiguous())

  def gated_packed(self):
    """[2F, d] rows interleaved per 32 (gate rows, then up rows), biases."""
    def build():
      c, d, f = self.w_shape
      assert c == 2
      wt = self.w.transpose(1, 2)                      # [2, F, d]
      w = torch.stack([wt[0].reshape(f // 32, 32, d),
                       wt[1].reshape(f // 32, 32, d)], dim=1)
      return (w.reshape(2 * f, d).contiguous(), self.b[0].reshape(-1).contiguous(),
              self.b[1].reshape(-1).contiguous())
    return self._packed.get([self.w, self.b], build)

  def forward(self, x: torch.Tensor) -> torch.Tensor:
    self._check_eqn()
    wt = self.weights_nk()
    x2 = _flat(x)
    outs = [ops.linear(x2, wt[c], self.b[c].reshape(-1)) for c in
            range(self.w_shape[0])]
    return torch.stack(outs).view(self.w_shape[0], *x.shape[:-1],
                                  self.w_shape[-1])
