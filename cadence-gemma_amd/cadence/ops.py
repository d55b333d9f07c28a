"""torch.ops.cadence.* -- PyTorch-ROCm custom ops over the gfx950 C ABI.

Each op validates dtype / shape / layout (errors surface as RuntimeError,
like the reference's assert / ValueError sites), allocates its outputs
through the torch caching allocator, and enqueues the HIP kernels on the
current stream (graph-capturable: no host sync, no allocation in the C
layer).  Ops are registered for the CUDA (= HIP on ROCm) dispatch key only;
there is deliberately no CPU implementation.

Thin Python helpers below the registrations (`linear`, `rmsnorm`, ...) are
what the modules call; they route through `torch.ops.cadence`.
"""

from __future__ import annotations

import contextlib
import ctypes
import math
import os
from typing import NamedTuple

import torch

from . import _lib

_BF16 = torch.bfloat16
_F32 = torch.float32
_I32 = torch.int32

_LIBDEF = torch.library.Library("cadence", "DEF")


def _reg(schema: str):
  name = schema.split("(")[0]
  _LIBDEF.define(schema)

  def deco(fn):
    _LIBDEF.impl(name, fn, "CUDA")
    return fn
  return deco


def _p(t):
  return None if t is None else t.data_ptr()


def _s(t: torch.Tensor):
  return torch.cuda.current_stream(t.device).cuda_stream


def _need(cond: bool, msg: str):
  if not cond:
    raise RuntimeError(msg)


def _mat(t: torch.Tensor, name: str, dtype=_BF16) -> int:
  """Validates a row-major 2-D (view) operand and returns its leading dim."""
  _need(t.dim() == 2, f"{name}: expected 2-D, got {tuple(t.shape)}")
  _need(t.dtype == dtype, f"{name}: expected {dtype}, got {t.dtype}")
  _need(t.stride(1) == 1, f"{name}: last dim must be contiguous")
  return t.stride(0)


class KernelTimer:
  """HIP-event timing of selected kernels on the stream they run on.

  Off by default.  When enabled (bench.py), each timed op brackets its
  launch(es) with two events on the current stream and records the
  algorithmic work of that launch; `summary()` syncs and returns per-kernel
  launch counts, average duration and average work.  Never records while a
  graph is being captured.  Events come from a pool created by `reset()`
  (creating them per launch costs host time inside the timed region), and
  `sample` = k times a seeded random 1/k of the launches: each event record
  costs the stream ~2-3 us, so timing every launch would slow the timed
  steps by ~2 %.
  """

  def __init__(self):
    self.enabled = False
    self.records: dict[str, list] = {}
    self.scope = ""
    self._pool: list = []
    self._next = 0
    self.sample = 1
    self._rng = None

  def reset(self, pool: int = 0, sample: int = 1, seed: int = 0):
    import random
    self.records = {}
    self._next = 0
    self.sample = max(1, sample)
    self._rng = random.Random(seed)
    if pool > len(self._pool):
      self._pool += [torch.cuda.Event(enable_timing=True)
                     for _ in range(pool - len(self._pool))]

  def _event(self):
    if self._next < len(self._pool):
      ev = self._pool[self._next]
    else:
      ev = torch.cuda.Event(enable_timing=True)
      self._pool.append(ev)
    self._next += 1
    return ev

  @contextlib.contextmanager
  def scoped(self, suffix: str):
    """Records inside get `suffix` appended to their key (the ViT towers run
    on two streams, so their per-launch event windows include time shared
    with the other tower: kept apart from the single-stream launches)."""
    prev, self.scope = self.scope, suffix
    try:
      yield
    finally:
      self.scope = prev

  def start(self, t: torch.Tensor):
    if not self.enabled or torch.cuda.is_current_stream_capturing():
      return None
    if self.sample > 1 and self._rng.randrange(self.sample):
      return None
    ev = self._event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev

  def stop(self, ev, key: str, work: float, t: torch.Tensor):
    if ev is None:
      return
    end = self._event()
    end.record(torch.cuda.current_stream(t.device))
    if not isinstance(work, torch.Tensor):
      work = float(work)
    self.records.setdefault(key + self.scope, []).append((ev, end, work))

  def summary(self) -> dict[str, dict]:
    torch.cuda.synchronize()
    out = {}
    for key, recs in self.records.items():
      ms = [a.elapsed_time(b) for a, b, _ in recs]
      work = [float(w) for _, _, w in recs]   # device scalars sync here
      out[key] = dict(launches=len(recs), total_ms=sum(ms),
                      avg_ms=sum(ms) / len(ms), avg_work=sum(work) / len(work),
                      total_work=sum(work))
    return out


TIMER = KernelTimer()


def _tile(M: int) -> bool:
  return M > 64


def _big_key(epi: str, M: int, N: int, K: int, groups: int = 1) -> str:
  """The rocprof name of the prefill GEMM kernel a launch runs:
  gemm_w4_kernel<Epi, MR> or gemm_big_kernel<Epi, P8, MR> (tile height
  32 MR, cadence_gemm_tile_rows; engine from cadence_gemm_engine)."""
  lib = _lib.load()
  rows = lib.cadence_gemm_tile_rows(M, N, K, groups)
  p8 = 1 if K % 128 == 0 else 0
  sk = lib.cadence_gemm_big_splits(M, N, K, groups)
  if sk > 1:   # split-K launch pair: partial GEMM + the epilogue's reduce
    return f"gemm_big_kernel<EpiPartial, {p8}, {rows // 32}> + splitk_reduce<{epi}> (split {sk})"
  if lib.cadence_gemm_engine(M, N, K, groups):
    return f"gemm_w4_kernel<{epi}, {rows // 32}>"
  return f"gemm_big_kernel<{epi}, {p8}, {rows // 32}>"


_COUNTERS: dict[tuple, torch.Tensor] = {}


def _counters(dev: torch.device, n: int):
  """Zeroed int32 arrival counters for the in-kernel split combines (kernels
  leave them at zero), one buffer per (device, stream): launches on one
  stream run in order, launches on two streams may overlap and must not
  share counters.  None while capturing before first use on that stream."""
  idx = dev.index if dev.index is not None else torch.cuda.current_device()
  key = (idx, torch.cuda.current_stream(idx).cuda_stream)
  buf = _COUNTERS.get(key)
  if buf is None or buf.numel() < n:
    if torch.cuda.is_current_stream_capturing():
      return None
    buf = torch.zeros(max(n, 4096), dtype=torch.int32, device=dev)
    _COUNTERS[key] = buf
  return buf


_WAIT_ERR: dict[int, torch.Tensor] = {}


def wait_err(dev: torch.device):
  """int32 flag a launch with an inter-workgroup wait sets to 1 if a wait
  gave up (never expected; tests read it), one per device.  None while
  capturing before first use."""
  idx = dev.index if dev.index is not None else torch.cuda.current_device()
  buf = _WAIT_ERR.get(idx)
  if buf is None:
    if torch.cuda.is_current_stream_capturing():
      return None
    buf = _WAIT_ERR[idx] = torch.zeros(1, dtype=torch.int32, device=dev)
  return buf


def _copy_region(dst: torch.Tensor, src: torch.Tensor):
  """(rows, row_bytes, src_stride, dst_stride) of a dst <- src copy whose
  views are each [rows, contiguous rest] (a whole contiguous tensor is one
  row), or None when the layout does not fit that form."""
  if dst.shape != src.shape or dst.dtype != src.dtype or dst.device != src.device:
    return None
  es = dst.element_size()
  if dst.is_contiguous() and src.is_contiguous():
    return 1, dst.numel() * es, 0, 0
  if dst.dim() < 2 or not (dst[0].is_contiguous() and src[0].is_contiguous()):
    return None
  return dst.shape[0], dst[0].numel() * es, src.stride(0) * es, dst.stride(0) * es


def copy_batched_(pairs) -> None:
  """dst.copy_(src) for every (dst, src) pair on the current stream, the
  row-strided ones batched into cadence_copy_batched launches (one per 32
  regions) instead of one copy kernel each; pairs that do not fit its
  layout (or 4-byte granularity) fall back to Tensor.copy_."""
  descs = []
  dev = None
  for dst, src in pairs:
    reg = _copy_region(dst, src) if dst.is_cuda else None
    if reg is None or reg[1] % 4 or reg[2] % 4 or reg[3] % 4 or \
        dst.data_ptr() % 4 or src.data_ptr() % 4:
      dst.copy_(src)
      continue
    if reg[0] * reg[1] == 0:
      continue
    dev = dst
    descs.append(_lib.CopyDesc(src.data_ptr(), dst.data_ptr(), *reg))
  if descs:
    arr = (_lib.CopyDesc * len(descs))(*descs)
    _lib.check(_lib.load().cadence_copy_batched(arr, len(descs), _s(dev)),
               "copy_batched")


def claim_counters(stream: torch.cuda.Stream, owner) -> None:
  """Hands the counter buffer of the capture `stream` over to `owner` (a
  captured decode graph, whose kernels hold its raw pointer) and removes it
  from the per-stream table.  The graph is replayed on other streams (a
  lane, the caller's), while torch's stream pool hands the capture stream's
  handle out again (32 handles, round robin): an eager launch on that handle
  must not find the graph's buffer, or its split combines would share
  arrival counters with a concurrent replay.  After the hand-over the next
  use of the handle allocates a fresh zeroed buffer."""
  key = (stream.device.index, stream.cuda_stream)
  buf = _COUNTERS.pop(key, None)
  if buf is not None:
    owner._cadence_counters = buf


def _ws(M: int, N: int, K: int, groups: int, like: torch.Tensor):
  n = _lib.load().cadence_gemm_workspace_bytes(M, N, K, groups)
  if n == 0:
    return None, 0
  return torch.empty(n, dtype=torch.uint8, device=like.device), n


# ------------------------------------------------------ packed decode rows



class PackedRows(NamedTuple):
  """M <= 32 activation rows in the decode fragment layout
  (include/cadence_kernels.h "Decode activation layout"): what the decode
  producers (RMSNorm, gated GELU, RG-LRU step, decode attention) emit and
  the decode GEMVs consume, so each wave's activation load is 1 KiB of
  contiguous bytes.  `data` is a flat bf16 tensor of k * 16 * ceil(m/16).

  With `norm` set (a layers.RMSNorm), `data` holds the rows BEFORE that
  norm (cadence_gemm_linear_residual_rows) and `src` the same rows
  row-major: the norm-aware decode GEMVs (linear_conv1d_, qkv_rope_decode,
  gated_gelu) apply it on load; any other consumer gets normalised rows
  from `normalised()`."""
  data: torch.Tensor
  m: int
  k: int
  norm: object = None
  src: torch.Tensor | None = None

  def normalised(self) -> "PackedRows":
    if self.norm is None:
      return self
    return PackedRows(ops.rmsnorm(self.src, self.norm.scale, self.norm.eps, True),
                      self.m, self.k)

  @property
  def shape(self):
    return (self.m, self.k)

  @property
  def device(self):
    return self.data.device

  @property
  def dtype(self):
    return self.data.dtype

  def unpack(self) -> torch.Tensor:
    """Row-major [m, k] copy (tests / debugging)."""
    mt = -(-self.m // 16)
    x = self.data.view(self.k // 32, mt, 4, 16, 8).permute(1, 3, 0, 2, 4)
    return x.reshape(mt * 16, self.k)[: self.m]


def want_packed(m: int, k: int) -> bool:
  return 0 < m <= 32 and k % 32 == 0


def packed_empty(m: int, k: int, device) -> torch.Tensor:
  return torch.empty(k * 16 * (-(-m // 16)), dtype=_BF16, device=device)


def pack_rows(x: torch.Tensor) -> PackedRows:
  """Row-major [m, k] -> PackedRows (torch ops; tests and one-off use)."""
  m, k = x.shape
  mt = -(-m // 16)
  xp = torch.zeros(mt * 16, k, dtype=x.dtype, device=x.device)
  xp[:m] = x
  data = xp.view(mt, 16, k // 32, 4, 8).permute(2, 0, 3, 1, 4).contiguous().view(-1)
  return PackedRows(data, m, k)


def _arows(a, name: str):
  """(tensor to pass, lda, M, K) of a GEMM A operand: a row-major view or
  PackedRows (lda 0)."""
  if isinstance(a, PackedRows):
    a = a.normalised()
    _need(a.data.dtype == _BF16 and a.data.is_contiguous(), f"{name}: packed rows")
    return a.data, 0, a.m, a.k
  lda = _mat(a, name)
  return a, lda, a.shape[0], a.shape[1]


# ------------------------------------------------------------------- GEMMs

# ------------------------------------------------- decode weight layout

def pack_decode(w: torch.Tensor) -> torch.Tensor:
  """Fragment-packed copy of a [.., N, K] weight (cadence_kernels.h "Decode
  weight layout"): per 16-row x 32-column tile, the 64 MFMA lanes' 16-B
  fragments back to back, so decode GEMMs stream 1 KiB per wave load."""
  *g, n, k = w.shape
  _need(n % 16 == 0 and k % 32 == 0, "decode packing needs N % 16, K % 32")
  return (w.reshape(*g, n // 16, 16, k // 32, 4, 8).movedim(-4, -2)
          .contiguous().view(w.shape))


def decode_weight(w: torch.Tensor):
  """The cached fragment-packed copy of `w` for M <= 32 launches (rebuilt
  when `w` changes), or None when it cannot be packed or would be built
  inside a graph capture."""
  if w.dim() < 2 or w.shape[-2] % 16 or w.shape[-1] % 32 or not w.is_cuda:
    return None
  c = getattr(w, "_cadence_decode", None)
  key = (w.data_ptr(), w._version)
  if c is not None and c[0] == key:
    return c[1]
  if torch.cuda.is_current_stream_capturing():
    return None
  with torch.no_grad():
    packed = pack_decode(w.detach())
  w._cadence_decode = (key, packed)
  return packed


def fold_norm(w: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
  """bf16(w[..., k] * bf16(1 + scale[k])): an RMSNorm's scale folded into the
  columns of the weight that consumes its output (cadence_kernels.h
  "Deferred RMSNorm"); the same two roundings as torch on bf16 tensors."""
  c = scale.detach() + 1.0
  return w.detach() * c


def decode_weight_norm(w: torch.Tensor, norm):
  """The cached fragment-packed copy of fold_norm(w, norm.scale) for decode
  GEMVs that normalise on load (rebuilt when `w` or the scale changes), or
  None when it cannot be packed or would be built inside a graph capture."""
  if w.dim() < 2 or w.shape[-2] % 16 or w.shape[-1] % 32 or not w.is_cuda:
    return None
  sc = norm.scale
  c = getattr(w, "_cadence_decode_norm", None)
  key = (w.data_ptr(), w._version, sc.data_ptr(), sc._version)
  if c is not None and c[0] == key:
    return c[1]
  if torch.cuda.is_current_stream_capturing():
    return None
  with torch.no_grad():
    packed = pack_decode(fold_norm(w, sc))
  w._cadence_decode_norm = (key, packed)
  return packed


def _wld(w, packed: bool, name: str) -> int:
  if packed:
    _need(w.is_contiguous() and w.dtype == _BF16, f"{name}: packed layout")
    return 0
  return _mat(w, name)


@_reg("gemm_linear_(Tensor a, Tensor w, Tensor? bias, Tensor? resid, "
      "Tensor(a!) out, int act, int row_div, int row_mul, int row_off, "
      "bool w_packed=False, int a_rows=-1) -> ()")
def _gemm_linear(a, w, bias, resid, out, act, row_div, row_mul, row_off,
                 w_packed=False, a_rows=-1):
  """a_rows >= 0: `a` is PackedRows data of a_rows rows (lda 0)."""
  ldw, ldo = _wld(w, w_packed, "w"), _mat(out, "out")
  N, K = w.shape[0], w.shape[1]
  if a_rows >= 0:
    lda, M = 0, a_rows
    _need(a.numel() == K * 16 * (-(-M // 16)), "a: packed rows size")
  else:
    lda = _mat(a, "a")
    M, K = a.shape
  _need(w.shape[1] == K, f"K mismatch {K} vs {w.shape[1]}")
  ldr = 0
  if resid is not None:
    ldr = _mat(resid, "resid")
  if bias is not None:
    _need(bias.numel() == N and bias.dtype == _BF16, "bias shape/dtype")
  ws, nws = _ws(M, N, K, 1, a)
  ev = TIMER.start(a) if _tile(M) else None
  _lib.check(_lib.load().cadence_gemm_linear(
      _p(a), lda, _p(w), ldw, _p(bias), _p(resid), ldr, _p(out), ldo, M, N, K,
      act, row_div, row_mul, row_off, _p(ws), nws, _s(a)), "gemm_linear")
  if ev is not None:
    TIMER.stop(ev, _big_key(f"EpiLinearA<{act}>", M, N, K), 2.0 * M * N * K, a)


@_reg("gemm_linear_conv1d_(Tensor a, Tensor w, Tensor? bias, Tensor conv_w, "
      "Tensor conv_b, Tensor(a!) conv_state, bool w_packed=False, "
      "int a_rows=-1, bool norm=False, float norm_eps=0.0) -> Tensor")
def _gemm_linear_conv1d(a, w, bias, conv_w, conv_b, conv_state, w_packed=False,
                        a_rows=-1, norm=False, norm_eps=0.0):
  """Decode y|x projection fused with the x branch's Conv1D step: returns
  [M, 2E] = (y, conv1d_step(x)); `conv_state` [M, TW-1, E] advances in place."""
  ldw = _wld(w, w_packed, "w")
  N, K = w.shape[0], w.shape[1]
  if a_rows >= 0:
    lda, M = 0, a_rows
    _need(a.numel() == K * 16 * (-(-M // 16)), "a: packed rows size")
  else:
    lda = _mat(a, "a")
    M, K = a.shape
  TW, E = conv_w.shape
  _need(N == 2 * E and conv_b.numel() == E, "conv width vs projection width")
  _need(conv_state.is_contiguous() and conv_state.dtype == _BF16 and
        tuple(conv_state.shape) == (M, TW - 1, E), "conv state")
  if bias is not None:
    _need(bias.numel() == N and bias.dtype == _BF16, "bias shape/dtype")
  out = torch.empty(M, N, dtype=_BF16, device=a.device)
  _lib.check(_lib.load().cadence_gemm_linear_conv1d(
      _p(a), lda, _p(w), ldw, _p(bias), _p(out), N, M, N, K, E,
      _p(conv_w.contiguous()), _p(conv_b.contiguous()), _p(conv_state), TW,
      _norm_flag(norm, lda), float(norm_eps), _s(a)),
      "gemm_linear_conv1d")
  return out


@_reg("recurrent_decode_front(Tensor a, int a_rows, Tensor w, Tensor? bias, "
      "Tensor conv_w, Tensor conv_b, Tensor(a!) conv_state, Tensor wg, "
      "Tensor bias_x, Tensor bias_a, Tensor softplus_a, Tensor segment_pos, "
      "Tensor(b!) h, Tensor(c!) counters, Tensor(d!) err, bool norm=False, "
      "float norm_eps=0.0) -> (Tensor, Tensor)")
def _recurrent_decode_front(a, a_rows, w, bias, conv_w, conv_b, conv_state, wg, bias_x,
                            bias_a, softplus_a, segment_pos, h, counters, err, norm=False,
                            norm_eps=0.0):
  """Decode recurrent-block front in one launch: gemm_linear_conv1d_ (packed
  rows, decode-packed w) then rglru_step_ on its output (gate = y branch,
  decode-packed wg, packed y).  Returns (yx [M, 2E], y packed rows);
  conv_state and h advance in place."""
  M = a_rows
  N, K = w.shape[0], w.shape[1]
  TW, E = conv_w.shape
  H, two_bw, bw = wg.shape
  _need(TW == 4 and N == 2 * E and conv_b.numel() == E, "conv width vs projection width")
  _need(two_bw == 2 * bw and H * bw == E, "gate weight shape")
  _need(a.numel() == K * 16 * (-(-M // 16)), "a: packed rows size")
  _need(conv_state.is_contiguous() and conv_state.dtype == _BF16 and
        tuple(conv_state.shape) == (M, TW - 1, E), "conv state")
  _need(h.dtype == _F32 and h.is_contiguous() and tuple(h.shape) == (M, E),
        "h: [M, E] fp32 contiguous")
  _need(segment_pos.dtype == _I32 and segment_pos.numel() == M, "segment_pos")
  _need(counters.dtype == _I32 and counters.numel() >= 64 * H and
        err.dtype == _I32 and err.numel() >= 1, "counters / err")
  if bias is not None:
    _need(bias.numel() == N and bias.dtype == _BF16, "bias shape/dtype")
  lib = _lib.load()
  _need(lib.cadence_recurrent_decode_front_plan(M, E, K, H, bw) == 1,
        "recurrent_decode_front: shape outside its plan")
  yx = torch.empty(M, N, dtype=_BF16, device=a.device)
  y = packed_empty(M, E, a.device)
  _lib.check(lib.cadence_recurrent_decode_front(
      _p(a), _p(w), _p(bias), _p(yx), M, E, K, _p(conv_w.contiguous()),
      _p(conv_b.contiguous()), _p(conv_state), 1 if norm else 0, float(norm_eps),
      _p(wg), _p(bias_x), _p(bias_a), _p(softplus_a), _p(segment_pos.contiguous()),
      _p(h), _p(y), H, bw, _p(counters), _p(err), _s(a)), "recurrent_decode_front")
  return yx, y


@_reg("gemm_linear_rmsnorm(Tensor a, Tensor w, Tensor? bias, Tensor? resid, "
      "Tensor scale, float eps, bool w_packed=False, int a_rows=-1, "
      "bool norm_packed=False) -> (Tensor, Tensor)")
def _gemm_linear_rmsnorm(a, w, bias, resid, scale, eps, w_packed=False,
                         a_rows=-1, norm_packed=False):
  """(out, rmsnorm(out)): out = a . w^T + bias (+ resid).  a_rows >= 0: `a`
  is PackedRows data; norm_packed: rmsnorm(out) as PackedRows data."""
  ldw = _wld(w, w_packed, "w")
  N, K = w.shape[0], w.shape[1]
  if a_rows >= 0:
    lda, M = 0, a_rows
  else:
    lda = _mat(a, "a")
    M, K = a.shape
  ldr = _mat(resid, "resid") if resid is not None else 0
  out = torch.empty(M, N, dtype=_BF16, device=a.device)
  nout = (packed_empty(M, N, a.device) if norm_packed else
          torch.empty(M, N, dtype=_BF16, device=a.device))
  lib = _lib.load()
  nws = max(lib.cadence_gemm_rmsnorm_workspace_bytes(M, N, K),
            lib.cadence_gemm_workspace_bytes(M, N, K, 1))
  ws = torch.empty(nws, dtype=torch.uint8, device=a.device) if nws else None
  if _tile(M) and TIMER.enabled:
    # the same two launches cadence_gemm_linear_rmsnorm makes for M > 32,
    # as two calls so the GEMM is timed on its own
    ev = TIMER.start(a)
    _lib.check(lib.cadence_gemm_linear(
        _p(a), lda, _p(w), ldw, _p(bias), _p(resid), ldr, _p(out), N, M, N, K,
        0, M, 0, 0, _p(ws), nws, _s(a)), "gemm_linear")
    TIMER.stop(ev, _big_key("EpiLinearA<0>", M, N, K), 2.0 * M * N * K, a)
    _lib.check(lib.cadence_rmsnorm(_p(out), N, _p(scale), _p(nout),
                                   0 if norm_packed else N, M, N, float(eps), _s(a)),
               "rmsnorm")
    return out, nout
  _lib.check(lib.cadence_gemm_linear_rmsnorm(
      _p(a), lda, _p(w), ldw, _p(bias), _p(resid), ldr, _p(out), N, M, N, K,
      _p(scale), float(eps), _p(nout), 0 if norm_packed else N, _p(ws), nws,
      _s(a)),
      "gemm_linear_rmsnorm")
  return out, nout


def _norm_flag(norm: bool, lda: int) -> int:
  """Normalise-on-load flag of a decode GEMV (needs packed rows)."""
  _need(not norm or lda == 0, "norm on load needs packed rows")
  return 1 if norm else 0


@_reg("gemm_linear_residual_rows(Tensor a, Tensor w, Tensor? bias, "
      "Tensor? resid, bool w_packed=False, int a_rows=-1) -> (Tensor, Tensor)")
def _gemm_linear_residual_rows(a, w, bias, resid, w_packed=False, a_rows=-1):
  """Decode (M <= 32) residual GEMM: (out = a . w^T + bias + resid, the same
  rows as PackedRows data, unnormalised) -- the consumer applies the norm.
  Split-K combined in-kernel (arrival counters of the current stream)."""
  ldw = _wld(w, w_packed, "w")
  N, K = w.shape[0], w.shape[1]
  if a_rows >= 0:
    lda, M = 0, a_rows
    _need(a.numel() == K * 16 * (-(-M // 16)), "a: packed rows size")
  else:
    lda = _mat(a, "a")
    M, K = a.shape
  _need(w.shape[1] == K, f"K mismatch {K} vs {w.shape[1]}")
  ldr = _mat(resid, "resid") if resid is not None else 0
  if bias is not None:
    _need(bias.numel() == N and bias.dtype == _BF16, "bias shape/dtype")
  lib = _lib.load()
  nws = lib.cadence_gemm_rmsnorm_workspace_bytes(M, N, K)
  _need(nws > 0 and M <= 32, "residual rows: decode shapes only")
  cnt = _counters(a.device, N // 16)
  _need(cnt is not None, "residual rows: no arrival counters on this stream")
  out = torch.empty(M, N, dtype=_BF16, device=a.device)
  rows = packed_empty(M, N, a.device)
  ws = torch.empty(nws, dtype=torch.uint8, device=a.device)
  _lib.check(lib.cadence_gemm_linear_residual_rows(
      _p(a), lda, _p(w), ldw, _p(bias), _p(resid), ldr, _p(out), N, _p(rows), M,
      N, K, _p(ws), nws, _p(cnt), _s(a)), "gemm_linear_residual_rows")
  return out, rows


@_reg("gated_gelu(Tensor a, Tensor w_packed, Tensor bias_gate, "
      "Tensor bias_up, bool decode_layout=False, int a_rows=-1, "
      "bool out_packed=False, bool norm=False, float norm_eps=0.0) -> Tensor")
def _gated_gelu(a, w_packed, bias_gate, bias_up, decode_layout=False, a_rows=-1,
                out_packed=False, norm=False, norm_eps=0.0):
  F, K = w_packed.shape[0] // 2, w_packed.shape[1]
  if a_rows >= 0:
    lda, M = 0, a_rows
  else:
    lda = _mat(a, "a")
    M = a.shape[0]
    _need(a.shape[1] == K, "a / w_packed K mismatch")
  _need(w_packed.is_contiguous(), "w_packed")
  out = (packed_empty(M, F, a.device) if out_packed else
         torch.empty(M, F, dtype=_BF16, device=a.device))
  ws, nws = _ws(M, 2 * F, K, 1, a)
  ev = TIMER.start(a) if _tile(M) else None
  _lib.check(_lib.load().cadence_gemm_gated_gelu(
      _p(a), lda, _p(w_packed), 0 if decode_layout else K, _p(bias_gate),
      _p(bias_up), _p(out), 0 if out_packed else F, M, F, K, _p(ws), nws,
      _norm_flag(norm, lda), float(norm_eps), _s(a)),
      "gated_gelu")
  if ev is not None:
    TIMER.stop(ev, _big_key("EpiGatedGelu", M, 2 * F, K), 4.0 * M * F * K, a)
  return out


@_reg("rglru_gates(Tensor x, Tensor w_packed, Tensor bias_x, Tensor bias_a, "
      "Tensor softplus_a, Tensor segment_pos, bool decode_layout=False) "
      "-> (Tensor, Tensor)")
def _rglru_gates(x, w_packed, bias_x, bias_a, softplus_a, segment_pos,
                 decode_layout=False):
  ldx = _mat(x, "x")
  M, E = x.shape
  H, two_bw, bw = w_packed.shape
  _need(two_bw == 2 * bw and H * bw == E, "w_packed shape")
  _need(segment_pos.dtype == _I32 and segment_pos.numel() == M, "segment_pos")
  a = torch.empty(M, E, dtype=_BF16, device=x.device)
  nx = torch.empty(M, E, dtype=_BF16, device=x.device)
  ws, nws = _ws(M, 2 * bw, bw, H, x)
  ev = TIMER.start(x) if _tile(M) else None
  _lib.check(_lib.load().cadence_rglru_gates(
      _p(x), ldx, _p(w_packed), 0 if decode_layout else bw, _p(bias_x),
      _p(bias_a), _p(softplus_a), _p(segment_pos.contiguous()), _p(a), _p(nx),
      E, M, H, bw, _p(ws), nws,
      _s(x)), "rglru_gates")
  if ev is not None:
    if _lib.load().cadence_rglru_gates_stream_plan(
        _p(x), ldx, _p(w_packed), 0 if decode_layout else bw, E, M, bw):
      # the block-bound streaming kernel: priced on HBM bytes (x in, a and
      # normalised x out, the packed weights once)
      TIMER.stop(ev, f"rglru_gates_stream_kernel<{bw}>",
                 3.0 * M * E * 2 + w_packed.numel() * 2, x)
    else:
      TIMER.stop(ev, _big_key("EpiRglruGates", M, 2 * bw, bw, H),
                 2.0 * M * 2 * bw * bw * H, x)
  return a, nx


def rglru_scan_plan(x, gate, B, L, heads, bw) -> bool:
  """Host-only query: the fused gates + scan kernel takes these operands."""
  return bool(_lib.load().cadence_rglru_scan_plan(
      _p(x), x.stride(0), _p(gate), gate.stride(0) if gate is not None else 0,
      heads * bw, B, L, heads, bw))


@_reg("rglru_scan(Tensor x, Tensor w_packed, Tensor bias_x, Tensor bias_a, "
      "Tensor softplus_a, Tensor segment_pos, Tensor? h0, Tensor? gate, int B, "
      "int L) -> (Tensor, Tensor)")
def _rglru_scan(x, w_packed, bias_x, bias_a, softplus_a, segment_pos, h0, gate,
                B, L):
  """Prefill gates + scan in one launch (rglru_gates then rnn_scan, bitwise):
  returns (bf16(h) [* gate] [B * L, E], h_last [B, E] fp32)."""
  ldx = _mat(x, "x")
  M, E = x.shape
  H, two_bw, bw = w_packed.shape
  _need(two_bw == 2 * bw and H * bw == E and M == B * L, "w_packed / x shape")
  # the kernel reads w_packed as a dense row-major [H][2 bw][bw] array (no
  # leading dimension is passed) and the three gate vectors by channel
  _need(w_packed.is_contiguous() and w_packed.dtype == _BF16,
        "w_packed: contiguous bf16 [H, 2 bw, bw]")
  for name, v in (("bias_x", bias_x), ("bias_a", bias_a), ("softplus_a", softplus_a)):
    _need(v.dtype == _BF16 and v.numel() == E and v.is_contiguous(),
          f"{name}: contiguous bf16 [E]")
  _need(segment_pos.dtype == _I32 and segment_pos.numel() == M, "segment_pos")
  if gate is not None:
    _need(tuple(gate.shape) == (M, E), "gate: [B * L, E]")
  ldg = _mat(gate, "gate") if gate is not None else 0
  if h0 is not None:
    _need(h0.dtype == _F32 and h0.is_contiguous() and tuple(h0.shape) == (B, E),
          "h0: [B, E] fp32")
  out = torch.empty(M, E, dtype=_BF16, device=x.device)
  h_last = torch.empty(B, E, dtype=_F32, device=x.device)
  ev = TIMER.start(x)
  _lib.check(_lib.load().cadence_rglru_scan(
      _p(x), ldx, _p(w_packed), _p(bias_x), _p(bias_a), _p(softplus_a),
      _p(segment_pos.contiguous()), _p(h0), _p(gate), ldg, _p(out), E,
      _p(h_last), B, L, H, bw, _s(x)), "rglru_scan")
  # algorithmic HBM bytes: x (+ gate) in, y out (bf16 per element), the
  # packed gate weights once, fp32 state out (+ in), int32 positions
  nbytes = (M * E * (4 + (2 if gate is not None else 0)) + w_packed.numel() * 2
            + B * E * 4 * (2 if h0 is not None else 1) + M * 4)
  TIMER.stop(ev, f"rglru_scan_fused_kernel<{bw}>", nbytes, x)
  return out, h_last


@_reg("rglru_step_(Tensor x, Tensor w_packed, Tensor bias_x, Tensor bias_a, "
      "Tensor softplus_a, Tensor segment_pos, Tensor(a!) h, Tensor? gate, "
      "bool decode_layout=False, bool out_packed=False) -> Tensor")
def _rglru_step(x, w_packed, bias_x, bias_a, softplus_a, segment_pos, h, gate,
                decode_layout=False, out_packed=False):
  """Gate GEMM + chain + the T == 1 scan step; `h` [M, E] fp32 in place."""
  ldx = _mat(x, "x")
  M, E = x.shape
  H, two_bw, bw = w_packed.shape
  _need(two_bw == 2 * bw and H * bw == E, "w_packed shape")
  _need(segment_pos.dtype == _I32 and segment_pos.numel() == M, "segment_pos")
  _need(h.dtype == _F32 and h.is_contiguous() and tuple(h.shape) == (M, E),
        "h: [M, E] fp32 contiguous")
  ldg = _mat(gate, "gate") if gate is not None else 0
  y = (packed_empty(M, E, x.device) if out_packed else
       torch.empty(M, E, dtype=_BF16, device=x.device))
  ws, nws = _ws(M, 2 * bw, bw, H, x)
  _lib.check(_lib.load().cadence_rglru_step(
      _p(x), ldx, _p(w_packed), 0 if decode_layout else bw, _p(bias_x),
      _p(bias_a), _p(softplus_a), _p(segment_pos.contiguous()), _p(h),
      _p(gate), ldg, _p(y), 0 if out_packed else E, M, H, bw, _p(ws), nws,
      _s(x)), "rglru_step")
  return y


@_reg("vit_residual_(Tensor a, Tensor w, Tensor bias, Tensor? gamma, "
      "Tensor(a!) resid) -> ()")
def _vit_residual(a, w, bias, gamma, resid):
  lda, ldw = _mat(a, "a"), _mat(w, "w")
  ldr = _mat(resid, "resid", _F32)
  M, K = a.shape
  N = w.shape[0]
  ws, nws = _ws(M, N, K, 1, a)
  ev = TIMER.start(a) if _tile(M) else None
  _lib.check(_lib.load().cadence_gemm_vit_residual(
      _p(a), lda, _p(w), ldw, _p(bias), _p(gamma), _p(resid), ldr, M, N, K,
      _p(ws), nws, _s(a)), "vit_residual")
  if ev is not None:
    TIMER.stop(ev, _big_key("EpiVitResid", M, N, K), 2.0 * M * N * K, a)


@_reg("patch_embed_(Tensor patches, Tensor w, Tensor bias, Tensor pos, "
      "Tensor(a!) resid, int B, int P, int ntok, int prefix) -> ()")
def _patch_embed(patches, w, bias, pos, resid, B, P, ntok, prefix):
  ldp, ldw = _mat(patches, "patches"), _mat(w, "w")
  N, K = w.shape
  _need(resid.dtype == _F32 and resid.is_contiguous(), "resid")
  ws, nws = _ws(B * P, N, K, 1, patches)
  _lib.check(_lib.load().cadence_gemm_patch_embed(
      _p(patches), ldp, _p(w), ldw, _p(bias), _p(pos), _p(resid), B, P, ntok,
      prefix, N, K, _p(ws), nws, _s(patches)), "patch_embed")


@_reg("logits_argmax(Tensor x, Tensor embedding, float soft_cap, "
      "bool return_logits, bool decode_layout=False, int a_rows=-1) "
      "-> (Tensor, Tensor)")
def _logits_argmax(x, embedding, soft_cap, return_logits, decode_layout=False,
                   a_rows=-1):
  D = embedding.shape[1]
  if a_rows >= 0:
    ldx, M = 0, a_rows
  else:
    ldx = _mat(x, "x")
    M, D = x.shape
  V = embedding.shape[0]
  L = _lib.load()
  nscr = L.cadence_logits_scratch_bytes(M, V, D)
  scratch = torch.empty(nscr, dtype=torch.uint8, device=x.device)
  logits = torch.empty((M, V) if return_logits else (0,), dtype=_BF16,
                       device=x.device)
  nxt = torch.empty(M, dtype=_I32, device=x.device)
  _lib.check(L.cadence_logits_argmax(
      _p(x), ldx, _p(embedding), 0 if decode_layout else D, M, V, D,
      float(soft_cap), _p(logits) if return_logits else None, _p(nxt),
      _p(scratch), nscr,
      _s(x)), "logits_argmax")
  return logits, nxt


@_reg("logits_argmax_tail_(Tensor x, Tensor embedding, float soft_cap, bool decode_layout, "
      "int a_rows, Tensor(a!) tokens_out, Tensor(a!) step, Tensor(a!) positions, "
      "Tensor(a!) cur, Tensor(a!)? done, int eos_id, int pad_id, int eos_from, "
      "Tensor(a!) counter, Tensor table, float scale, Tensor(a!) x_out, "
      "Tensor(a!) packed_out) -> Tensor")
def _logits_argmax_tail(x, embedding, soft_cap, decode_layout, a_rows, tokens_out, step,
                        positions, cur, done, eos_id, pad_id, eos_from, counter, table,
                        scale, x_out, packed_out):
  """The decode step's greedy tail (cadence_logits_argmax_tail): logits ->
  argmax -> decode_advance bookkeeping -> the next step's input rows
  (`table` = the row-major embedding)."""
  D = embedding.shape[1]
  if a_rows >= 0:
    ldx, M = 0, a_rows
  else:
    ldx = _mat(x, "x")
    M, D = x.shape
  V = embedding.shape[0]
  for t, name in ((tokens_out, "tokens_out"), (step, "step"), (positions, "positions"),
                  (cur, "cur"), (counter, "counter")):
    _need(t.dtype == _I32 and t.is_contiguous(), f"{name} int32")
  _need(done is None or (done.dtype == _I32 and done.numel() == M + 1), "done int32[M + 1]")
  _need(tokens_out.dim() == 2 and tokens_out.shape[0] == M, "tokens_out [M, steps]")
  _need(tuple(x_out.shape) == (M, D) and want_packed(M, D) and
        packed_out.numel() == D * 16 * (-(-M // 16)), "x_out / packed_out rows")
  L = _lib.load()
  nscr = L.cadence_logits_scratch_bytes(M, V, D)
  scratch = torch.empty(nscr, dtype=torch.uint8, device=x.device)
  nxt = torch.empty(M, dtype=_I32, device=x.device)
  tail = _lib.DecodeTail(
      _p(tokens_out), tokens_out.stride(0), _p(step), _p(positions), _p(cur),
      _p(done) if done is not None else None, int(eos_id), int(pad_id), int(eos_from),
      _p(counter), _p(table), table.shape[0], float(scale), _p(x_out), _mat(x_out, "x_out"),
      _p(packed_out))
  _lib.check(L.cadence_logits_argmax_tail(
      _p(x), ldx, _p(embedding), 0 if decode_layout else D, M, V, D, float(soft_cap),
      _p(nxt), _p(scratch), nscr, ctypes.byref(tail), _s(x)), "logits_argmax_tail")
  return nxt


@_reg("gemm_logits(Tensor x, Tensor embedding, float soft_cap, "
      "bool decode_layout=False, int a_rows=-1) -> Tensor")
def _gemm_logits(x, embedding, soft_cap, decode_layout=False, a_rows=-1):
  D = embedding.shape[1]
  if a_rows >= 0:
    ldx, M = 0, a_rows
  else:
    ldx = _mat(x, "x")
    M, D = x.shape
  V = embedding.shape[0]
  out = torch.empty(M, V, dtype=_BF16, device=x.device)
  ws, nws = _ws(M, V, D, 1, x)
  _lib.check(_lib.load().cadence_gemm_logits(
      _p(x), ldx, _p(embedding), 0 if decode_layout else D, M, V, D,
      float(soft_cap), _p(out), V, _p(ws), nws, _s(x)), "gemm_logits")
  return out


# ------------------------------------------------------ norms / embedding

@_reg("rmsnorm(Tensor x, Tensor scale, float eps, bool out_packed=False) "
      "-> Tensor")
def _rmsnorm(x, scale, eps, out_packed=False):
  ldx = _mat(x, "x")
  out = (packed_empty(x.shape[0], x.shape[1], x.device) if out_packed else
         torch.empty(x.shape, dtype=_BF16, device=x.device))
  _lib.check(_lib.load().cadence_rmsnorm(
      _p(x), ldx, _p(scale), _p(out), 0 if out_packed else x.shape[1],
      x.shape[0], x.shape[1], float(eps), _s(x)), "rmsnorm")
  return out


@_reg("layernorm(Tensor x, Tensor weight, Tensor bias, float eps) -> Tensor")
def _layernorm(x, weight, bias, eps):
  ldx = _mat(x, "x", _F32)
  out = torch.empty(x.shape, dtype=_BF16, device=x.device)
  _lib.check(_lib.load().cadence_layernorm(
      _p(x), ldx, _p(weight), _p(bias), _p(out), x.shape[1], x.shape[0],
      x.shape[1], float(eps), _s(x)), "layernorm")
  return out


@_reg("embed_(Tensor tokens, Tensor embedding, float scale, Tensor(a!) out, "
      "int row_div, int row_mul, int row_off) -> ()")
def _embed(tokens, embedding, scale, out, row_div, row_mul, row_off):
  _need(tokens.dtype == _I32 and tokens.is_contiguous(), "tokens int32")
  ldo = _mat(out, "out")
  _lib.check(_lib.load().cadence_embed(
      _p(tokens), _p(embedding), _p(out), ldo, tokens.numel(),
      embedding.shape[1], embedding.shape[0], float(scale), row_div, row_mul,
      row_off,
      _s(tokens)), "embed")


@_reg("embed_packed_(Tensor tokens, Tensor embedding, float scale, Tensor(a!) out, "
      "Tensor(a!) packed) -> ()")
def _embed_packed(tokens, embedding, scale, out, packed):
  """The decode step's embedding, row-major into `out` and in the decode
  activation layout into `packed` (cadence_embed_packed)."""
  _need(tokens.dtype == _I32 and tokens.is_contiguous(), "tokens int32")
  ldo = _mat(out, "out")
  m, d = tokens.numel(), embedding.shape[1]
  _need(tuple(out.shape) == (m, d) and want_packed(m, d), "embed_packed: [m <= 32, d % 32]")
  _need(packed.dtype == _BF16 and packed.is_contiguous() and
        packed.numel() == d * 16 * (-(-m // 16)), "embed_packed: packed rows")
  _lib.check(_lib.load().cadence_embed_packed(
      _p(tokens), _p(embedding), _p(out), ldo, _p(packed), m, d, embedding.shape[0],
      float(scale), _s(tokens)), "embed_packed")


# -------------------------------------------------------- recurrent block

@_reg("conv1d(Tensor x, Tensor w, Tensor b, Tensor segment_pos, Tensor? cache, "
      "int B, int L, bool compat) -> (Tensor, Tensor)")
def _conv1d(x, w, b, segment_pos, cache, B, L, compat):
  ldx = _mat(x, "x")
  E = x.shape[1]
  TW = w.shape[0]
  out = torch.empty(B * L, E, dtype=_BF16, device=x.device)
  new_cache = torch.empty(B, TW - 1, E, dtype=_BF16, device=x.device)
  if cache is not None:
    _need(L == 1 and tuple(cache.shape) == (B, TW - 1, E), "conv cache shape")
    cache = cache.to(_BF16).contiguous()
  _lib.check(_lib.load().cadence_conv1d(
      _p(x), ldx, _p(w), _p(b), _p(segment_pos.contiguous()), _p(cache),
      _p(out), E, _p(new_cache), B, L, E, TW, int(compat), _s(x)), "conv1d")
  return out, new_cache


def _scan_workspace(B, L, E, device):
  """Stream-ordered workspace for the chunked scan (small batches), from the
  caching allocator; (None, 0) when the sequential kernel runs."""
  n = _lib.load().cadence_rnn_scan_workspace_bytes(B, L, E)
  if n <= 0:
    return None, 0
  return torch.empty(n, dtype=torch.uint8, device=device), n


@_reg("rnn_scan(Tensor x, Tensor a, Tensor? segment_pos, Tensor? h0, "
      "Tensor? gate, int B, int L) -> (Tensor, Tensor)")
def _rnn_scan(x, a, segment_pos, h0, gate, B, L):
  ldx, lda = _mat(x, "x"), _mat(a, "a")
  E = x.shape[1]
  ldg = _mat(gate, "gate") if gate is not None else 0
  if h0 is not None:
    _need(h0.dtype == _F32 and h0.is_contiguous(), "h0 fp32")
  out = torch.empty(B * L, E, dtype=_BF16, device=x.device)
  h_last = torch.empty(B, E, dtype=_F32, device=x.device)
  pos = segment_pos.contiguous() if segment_pos is not None else None
  ws, wsb = _scan_workspace(B, L, E, x.device)
  ev = TIMER.start(x) if L > 1 else None
  _lib.check(_lib.load().cadence_rnn_scan(
      _p(x), ldx, _p(a), lda, _p(pos), _p(h0), _p(gate), ldg, _p(out), E,
      _p(h_last), B, L, E, _p(ws), wsb, _s(x)), "rnn_scan")
  # algorithmic bytes: x, a (+ gate) in and y out as bf16 per element,
  # fp32 state out (+ in), int32 reset per token when given
  per_elem = 6 + (2 if gate is not None else 0)
  nbytes = (B * L * E * per_elem + B * E * 4 * (2 if h0 is not None else 1)
            + (B * L * 4 if pos is not None else 0))
  TIMER.stop(ev, "rnn_scan_chunk_kernel" if wsb else "rnn_scan_kernel", nbytes, x)
  return out, h_last


@_reg("conv1d_step_(Tensor x, Tensor w, Tensor b, Tensor(a!) state) -> Tensor")
def _conv1d_step(x, w, b, state):
  """Single-token Conv1D updating its [B, W-1, E] state in place."""
  ldx = _mat(x, "x")
  B, E = x.shape
  TW = w.shape[0]
  _need(state.is_contiguous() and state.dtype == _BF16 and
        tuple(state.shape) == (B, TW - 1, E), "conv state")
  out = torch.empty(B, E, dtype=_BF16, device=x.device)
  _lib.check(_lib.load().cadence_conv1d(
      _p(x), ldx, _p(w), _p(b), None, _p(state), _p(out), E, _p(state), B, 1,
      E, TW, 1, _s(x)), "conv1d_step")
  return out


@_reg("rnn_scan_(Tensor x, Tensor a, Tensor(a!) h, Tensor? gate, int B, "
      "int L) -> Tensor")
def _rnn_scan_inplace(x, a, h, gate, B, L):
  """Scan continuing from and updating the fp32 state `h` [B, E] in place."""
  ldx, lda = _mat(x, "x"), _mat(a, "a")
  E = x.shape[1]
  ldg = _mat(gate, "gate") if gate is not None else 0
  _need(h.dtype == _F32 and h.is_contiguous(), "h fp32")
  out = torch.empty(B * L, E, dtype=_BF16, device=x.device)
  ws, wsb = _scan_workspace(B, L, E, x.device)
  _lib.check(_lib.load().cadence_rnn_scan(
      _p(x), ldx, _p(a), lda, None, _p(h), _p(gate), ldg, _p(out), E, _p(h), B,
      L, E, _p(ws), wsb, _s(x)), "rnn_scan_")
  return out


# ---------------------------------------------------------------- attention

@_reg("segment_info(Tensor segment_pos) -> (Tensor, Tensor)")
def _segment_info(segment_pos):
  B, L = segment_pos.shape
  seg = torch.empty(B, L, dtype=_I32, device=segment_pos.device)
  start = torch.empty(B, L, dtype=_I32, device=segment_pos.device)
  _lib.check(_lib.load().cadence_segment_info(
      _p(segment_pos.contiguous()), _p(seg), _p(start), B, L,
      _s(segment_pos)), "segment_info")
  return seg, start


ROPE_TABLE_POSITIONS = 8192
_rope_tables: dict = {}


def rope_table(device: torch.device, hd: int) -> torch.Tensor:
  """Per-(device, head dim) bf16 sin/cos table for positions < 8192, built
  once by a kernel (never reallocated, so captured graphs stay valid)."""
  key = (str(device), hd)
  t = _rope_tables.get(key)
  if t is None:
    t = torch.empty(ROPE_TABLE_POSITIONS, 2, hd // 4, dtype=_BF16,
                    device=device)
    _lib.check(_lib.load().cadence_rope_table(
        _p(t), ROPE_TABLE_POSITIONS, hd, _s(t)), "rope_table")
    _rope_tables[key] = t
  return t


@_reg("rope_qkv(Tensor qkv, Tensor positions, int H, int hd, "
      "Tensor? table=None) -> (Tensor, Tensor, Tensor)")
def _rope_qkv(qkv, positions, H, hd, table=None):
  ld = _mat(qkv, "qkv")
  M = qkv.shape[0]
  q = torch.empty(M, H * hd, dtype=_BF16, device=qkv.device)
  k = torch.empty(M, hd, dtype=_BF16, device=qkv.device)
  v = torch.empty(M, hd, dtype=_BF16, device=qkv.device)
  tlen = table.shape[0] if table is not None else 0
  _lib.check(_lib.load().cadence_rope_qkv(
      _p(qkv), ld, _p(positions.contiguous()), _p(q), _p(k), _p(v), M, H, hd,
      _p(table), tlen, _s(qkv)), "rope_qkv")
  return q, k, v


@_reg("qkv_rope_decode(Tensor a, Tensor w_perm, Tensor positions, int H, int hd, "
      "Tensor? table, bool w_packed=False, int a_rows=-1, bool norm=False, "
      "float norm_eps=0.0) -> (Tensor, Tensor, Tensor)")
def _qkv_rope_decode(a, w_perm, positions, H, hd, table=None, w_packed=False,
                     a_rows=-1, norm=False, norm_eps=0.0):
  """Decode q|k|v GEMV + RoPE; `w_perm` rows as qkv_rope_permutation().
  norm: `a` is unnormalised packed rows and `w_perm` carries the norm scale
  (fold_norm); the rows' rsqrt is applied in-kernel."""
  ldw = _wld(w_perm, w_packed, "w_perm")
  N, K = w_perm.shape[0], w_perm.shape[1]
  _need(N == (H + 2) * hd, "w_perm rows")
  if a_rows >= 0:
    lda, M = 0, a_rows
    _need(a.numel() == K * 16 * (-(-M // 16)), "a: packed rows size")
  else:
    lda = _mat(a, "a")
    M = a.shape[0]
  _need(positions.dtype == _I32 and positions.numel() == M, "positions")
  q = torch.empty(M, H * hd, dtype=_BF16, device=a.device)
  k = torch.empty(M, hd, dtype=_BF16, device=a.device)
  v = torch.empty(M, hd, dtype=_BF16, device=a.device)
  tlen = table.shape[0] if table is not None else 0
  _lib.check(_lib.load().cadence_qkv_rope_decode(
      _p(a), lda, _p(w_perm), ldw, _p(positions.contiguous()), _p(q), _p(k), _p(v),
      M, H, hd, K, _p(table), tlen, _norm_flag(norm, lda), float(norm_eps),
      _s(a)), "qkv_rope_decode")
  return q, k, v


@_reg("qkv_rope_prefill(Tensor a, Tensor w_perm, Tensor positions, int H, int hd, "
      "Tensor? table) -> (Tensor, Tensor, Tensor)")
def _qkv_rope_prefill(a, w_perm, positions, H, hd, table=None):
  """Prompt-pass q|k|v GEMM with RoPE in its epilogue (one block-engine
  launch; qkv_rope_prefill_ok() says whether the shape's plan allows it)."""
  lda, ldw = _mat(a, "a"), _mat(w_perm, "w_perm")
  M, K = a.shape
  N = w_perm.shape[0]
  _need(N == (H + 2) * hd and w_perm.shape[1] == K, "w_perm shape")
  _need(positions.dtype == _I32 and positions.numel() == M, "positions")
  q = torch.empty(M, H * hd, dtype=_BF16, device=a.device)
  k = torch.empty(M, hd, dtype=_BF16, device=a.device)
  v = torch.empty(M, hd, dtype=_BF16, device=a.device)
  tlen = table.shape[0] if table is not None else 0
  ev = TIMER.start(a)
  _lib.check(_lib.load().cadence_qkv_rope_prefill(
      _p(a), lda, _p(w_perm), ldw, _p(positions.contiguous()), _p(q), _p(k), _p(v),
      M, H, hd, K, _p(table), tlen, _s(a)), "qkv_rope_prefill")
  if ev is not None:
    TIMER.stop(ev, _big_key("EpiRopeQKVBig", M, N, K), 2.0 * M * N * K, a)
  return q, k, v


def qkv_rope_prefill_ok(M: int, H: int, hd: int, K: int) -> bool:
  """The fused prefill q|k|v + RoPE launch covers this shape: block engine,
  one K split, not the 4-wave engine (host-side plan queries)."""
  N = (H + 2) * hd
  if M <= 64 or hd % 64 or N % 64 or K % 64:
    return False
  lib = _lib.load()
  return (lib.cadence_gemm_big_splits(M, N, K, 1) == 1 and
          lib.cadence_gemm_engine(M, N, K, 1) == 0)


def qkv_rope_permutation(H: int, hd: int, device=None) -> torch.Tensor:
  """Row order of cadence_qkv_rope_decode's weight: in each of the H + 1
  q / k heads, rows 2i, 2i + 1 <- dims i, i + hd/4 (i < hd/4)."""
  perm = torch.arange((H + 2) * hd)
  q4 = hd // 4
  i = torch.arange(q4)
  for h in range(H + 1):
    perm[h * hd + 2 * i] = h * hd + i
    perm[h * hd + 2 * i + 1] = h * hd + q4 + i
  return perm.to(device) if device is not None else perm


@_reg("local_attention(Tensor q, Tensor k, Tensor v, Tensor seg_id, "
      "Tensor seg_start, int B, int L, int H, int hd, int window) -> Tensor")
def _local_attention(q, k, v, seg_id, seg_start, B, L, H, hd, window):
  for t in (q, k, v):
    _need(t.is_contiguous() and t.dtype == _BF16, "q/k/v contiguous bf16")
  out = torch.empty(B * L, H * hd, dtype=_BF16, device=q.device)
  work = None
  if TIMER.enabled and not torch.cuda.is_current_stream_capturing():
    # algorithmic work = the visible (query, key) pairs only: 4 * H * hd
    # FLOP each (QK^T and PV), the segment / causal / window mask applied;
    # a device scalar computed outside the timed window, once per positions
    # tensor (every attention block of a forward shares it)
    pairs = _visible_pairs.get((seg_start.data_ptr(), window))
    if pairs is None:
      idx = torch.arange(L, device=q.device, dtype=torch.int64)
      lo = torch.maximum(seg_start.view(B, L).long(), idx - window)
      pairs = (idx - lo + 1).sum().double()
      _visible_pairs.clear()
      _visible_pairs[(seg_start.data_ptr(), window)] = pairs
    work = pairs * (4.0 * H * hd)
  ev = TIMER.start(q)
  _lib.check(_lib.load().cadence_local_attention(
      _p(q), _p(k), _p(v), _p(seg_id), _p(seg_start), _p(out), B, L, H, hd,
      window, _s(q)), "local_attention")
  if ev is not None:
    key = ("griffin_attn_kernel<256>" if hd == 256 and H <= 10 else
           f"flash_attn_kernel<{hd},0>")
    TIMER.stop(ev, key, work, q)
  return out


_visible_pairs: dict = {}


@_reg("kv_cache_fill(Tensor k, Tensor v, Tensor segment_pos, int window) -> "
      "(Tensor, Tensor, Tensor)")
def _kv_cache_fill(k, v, segment_pos, window):
  B, L = segment_pos.shape
  hd = k.shape[-1]
  ck = torch.empty(B, window, 1, hd, dtype=_BF16, device=k.device)
  cv = torch.empty(B, window, 1, hd, dtype=_BF16, device=k.device)
  nt = torch.empty(B, dtype=_I32, device=k.device)
  _lib.check(_lib.load().cadence_kv_cache_fill(
      _p(k), _p(v), _p(segment_pos.contiguous()), _p(ck), _p(cv), _p(nt), B,
      L, hd, window, _s(k)), "kv_cache_fill")
  return ck, cv, nt


@_reg("local_attention_cached(Tensor q, Tensor k, Tensor v, Tensor cache_k, "
      "Tensor cache_v, Tensor num_tokens, int B, int T, int H, int hd, "
      "int window) -> Tensor")
def _local_attention_cached(q, k, v, cache_k, cache_v, num_tokens, B, T, H, hd,
                            window):
  """T query rows against [cache ring | T new keys] (cache-mask semantics,
  modules.py:155-185); the caches are read, not updated."""
  for t in (q, k, v, cache_k, cache_v):
    _need(t.is_contiguous() and t.dtype == _BF16, "q/k/v/caches contiguous bf16")
  _need(num_tokens.dtype == _I32, "num_tokens int32")
  out = torch.empty(B * T, H * hd, dtype=_BF16, device=q.device)
  _lib.check(_lib.load().cadence_local_attention_cached(
      _p(q), _p(k), _p(v), _p(cache_k), _p(cache_v), _p(num_tokens), _p(out),
      B, T, H, hd, window, _s(q)), "local_attention_cached")
  return out


@_reg("kv_ring_update_(Tensor k, Tensor v, Tensor(a!) cache_k, "
      "Tensor(b!) cache_v, Tensor(c!) num_tokens, int window) -> ()")
def _kv_ring_update(k, v, cache_k, cache_v, num_tokens, window):
  B = num_tokens.numel()
  hd = k.shape[-1]
  _need(k.is_contiguous() and v.is_contiguous(), "k/v contiguous")
  _need(cache_k.is_contiguous() and cache_v.is_contiguous(), "cache layout")
  _lib.check(_lib.load().cadence_kv_ring_update(
      _p(k), _p(v), _p(cache_k), _p(cache_v), _p(num_tokens), B, hd, window,
      _s(k)), "kv_ring_update")


@_reg("local_attention_decode_(Tensor q, Tensor k_new, Tensor v_new, "
      "Tensor(a!) cache_k, Tensor(b!) cache_v, Tensor(c!) num_tokens, int H, "
      "bool out_packed=False) -> Tensor")
def _local_attention_decode(q, k_new, v_new, cache_k, cache_v, num_tokens, H,
                            out_packed=False):
  B = q.shape[0]
  hd = k_new.shape[-1]
  W = cache_k.shape[1]
  _need(cache_k.is_contiguous() and cache_v.is_contiguous(), "cache layout")
  _need(num_tokens.dtype == _I32, "num_tokens int32")
  out = (packed_empty(B, H * hd, q.device) if out_packed else
         torch.empty(B, H * hd, dtype=_BF16, device=q.device))
  lib = _lib.load()
  nws = lib.cadence_local_attention_decode_workspace_bytes(B, hd)
  ws = torch.empty(nws, dtype=torch.uint8, device=q.device)
  sems = _counters(q.device, B)
  _lib.check(lib.cadence_local_attention_decode(
      _p(q.contiguous()), _p(k_new.contiguous()), _p(v_new.contiguous()),
      _p(cache_k), _p(cache_v), _p(num_tokens), _p(out),
      0 if out_packed else H * hd, B, H, hd, W,
      _p(ws) if sems is not None else None, nws, _p(sems), _s(q)),
      "local_attention_decode")
  return out


# ------------------------------------------------------------- vision tower

@_reg("im2col_normalize(Tensor pixels, float[] mean, float[] std, int patch, "
      "int kpad) -> Tensor")
def _im2col(pixels, mean, std, patch, kpad):
  import ctypes
  _need(pixels.dtype == _F32 and pixels.is_contiguous(), "pixels fp32")
  B, C, S, S2 = pixels.shape
  _need(C == 3 and S == S2 and len(mean) == 3 and len(std) == 3,
        "pixels [B,3,S,S], 3 means / stds")
  g = S // patch
  out = torch.empty(B * g * g, kpad, dtype=_BF16, device=pixels.device)
  m3 = (ctypes.c_float * 3)(*[float(v) for v in mean])
  s3 = (ctypes.c_float * 3)(*[float(v) for v in std])
  _lib.check(_lib.load().cadence_im2col_normalize(
      _p(pixels), _p(out), kpad, B, S, patch, ctypes.cast(m3, ctypes.c_void_p),
      ctypes.cast(s3, ctypes.c_void_p), _s(pixels)), "im2col")
  return out


def resize_taps(in_size: int, size: int) -> int:
  """Pillow precompute_coeffs ksize for one image side (Resample.c):
  ceil(2 * max(in / S, 1)) * 2 + 1, in the same double arithmetic."""
  scale = float(in_size) / size
  return int(math.ceil(2.0 * max(scale, 1.0))) * 2 + 1


@_reg("resize_bicubic(Tensor images, Tensor meta, int S, int KS, int max_h, "
      "int max_w, int tmp_bytes) -> Tensor")
def _resize_bicubic(images, meta, S, KS, max_h, max_w, tmp_bytes):
  _need(images.dtype == torch.uint8 and images.dim() == 1
        and images.is_contiguous(), "images packed u8")
  _need(meta.dtype == torch.int64 and meta.dim() == 2 and meta.shape[1] == 4
        and meta.is_contiguous() and meta.device == images.device,
        "meta [B, 4] int64 on the images' device")
  B = meta.shape[0]
  KS = (KS + 3) // 4 * 4            # coefficient rows padded to whole fours
  out = torch.empty(B, 3, S, S, dtype=_F32, device=images.device)
  coef = torch.empty(B * 2 * S * (2 + KS), dtype=_I32, device=images.device)
  tmp = torch.empty(max(tmp_bytes, 1), dtype=torch.uint8, device=images.device)
  _lib.check(_lib.load().cadence_resize_bicubic(
      _p(images), images.numel(), _p(meta), B, S, KS, max_h, max_w, _p(coef),
      _p(tmp), tmp.numel(), _p(out), _s(images)), "resize_bicubic")
  return out


@_reg("vit_prefix_(Tensor tokens, Tensor(a!) resid, int B, int ntok, "
      "int prefix) -> ()")
def _vit_prefix(tokens, resid, B, ntok, prefix):
  _lib.check(_lib.load().cadence_vit_prefix(
      _p(tokens.contiguous()), _p(resid), B, ntok, prefix, resid.shape[-1],
      _s(resid)), "vit_prefix")


@_reg("vit_attention(Tensor qkv, int B, int N, int H, int hd) -> Tensor")
def _vit_attention(qkv, B, N, H, hd):
  _need(qkv.is_contiguous() and qkv.dtype == _BF16, "qkv contiguous bf16")
  if qkv.data_ptr() % 16:      # the kernels load 16-B rows (C-ABI contract)
    qkv = qkv.clone()
  out = torch.empty(B * N, H * hd, dtype=_BF16, device=qkv.device)
  ev = TIMER.start(qkv)
  _lib.check(_lib.load().cadence_vit_attention(
      _p(qkv), _p(out), B, N, H, hd, _s(qkv)), "vit_attention")
  TIMER.stop(ev, vit_attention_kernel_name(N, hd), 4.0 * B * H * N * N * hd, qkv)
  return out


def vit_attention_kernel_name(N: int, hd: int) -> str:
  """The rocprof name (template arguments folded into hd) of the kernel
  cadence_vit_attention runs for this shape (host-side plan query)."""
  k = _lib.load().cadence_vit_attention_kernel(N, hd)
  return {0: "vit_attn_kernel", 1: "vit_stream_attn_kernel",
          2: "vit_flash_attn_kernel"}.get(k, "vit_attention?") + f"<hd{hd}>"


@_reg("vit_features_(Tensor resid, Tensor(a!) out, int col_off, int B, "
      "int ntok, int prefix) -> ()")
def _vit_features(resid, out, col_off, B, ntok, prefix):
  ldo = _mat(out, "out")
  _lib.check(_lib.load().cadence_vit_features(
      _p(resid), _p(out), ldo, col_off, B, ntok, prefix, resid.shape[-1],
      _s(resid)), "vit_features")


@_reg("splice_positions(Tensor text_pos, int n_vis) -> Tensor")
def _splice_positions(text_pos, n_vis):
  B, T = text_pos.shape
  out = torch.empty(B, n_vis + T, dtype=_I32, device=text_pos.device)
  _lib.check(_lib.load().cadence_splice_positions(
      _p(text_pos.contiguous()), _p(out), B, T, n_vis, _s(text_pos)),
      "splice_positions")
  return out


@_reg("decode_advance_(Tensor next_token, Tensor(a!) tokens_out, "
      "Tensor(b!) step, Tensor(c!) positions, Tensor(d!)? cur=None, "
      "Tensor(e!)? done=None, int eos_id=-1, int pad_id=0, int eos_from=1) -> ()")
def _decode_advance(next_token, tokens_out, step, positions, cur=None,
                    done=None, eos_id=-1, pad_id=0, eos_from=1):
  B = next_token.numel()
  _need(tokens_out.dtype == _I32 and tokens_out.stride(1) == 1, "tokens_out")
  if cur is not None:
    _need(cur.dtype == _I32 and cur.is_contiguous() and cur.numel() == B, "cur")
  if done is not None:
    _need(done.dtype == _I32 and done.is_contiguous() and done.numel() == B + 1,
          "done must be int32[B + 1]")
  _lib.check(_lib.load().cadence_decode_advance(
      _p(next_token), _p(tokens_out), tokens_out.stride(0), _p(step),
      _p(positions), _p(cur), _p(done), int(eos_id), int(pad_id),
      int(eos_from), B, _s(next_token)), "decode_advance")


# ----------------------------------------------------------------- helpers

ops = torch.ops.cadence


def _a(x):
  """(tensor, a_rows) of an A operand: PackedRows -> (data, m), else (x, -1)."""
  if isinstance(x, PackedRows):
    x = x.normalised()
    return x.data, x.m
  return x, -1


def _an(x, w):
  """(tensor, a_rows, weight, norm) of the A operand of a norm-aware decode
  GEMV and the weight to stream: rows whose RMSNorm is still pending go as
  they are with the fragment-packed, norm-folded weight (norm = the RMSNorm
  module); otherwise (tensor, a_rows, decode_weight(w) or None, None)."""
  if isinstance(x, PackedRows) and x.norm is not None and x.k <= 2560:
    wf = decode_weight_norm(w, x.norm)
    if wf is not None:
      return x.data, x.m, wf, x.norm
  a, ar = _a(x)
  return a, ar, (decode_weight(w) if x.shape[0] <= 32 else None), None


def linear(x2d, w, bias=None, act=0, resid=None, out=None,
           row_map=None):
  """out = act(x2d . w^T + bias) (+ resid); w [N, K] (nn.Linear layout).
  `x2d` may be PackedRows (decode rows)."""
  M = x2d.shape[0]
  N = w.shape[0]
  if out is None:
    out = torch.empty(M, N, dtype=_BF16, device=x2d.device)
  div, mul, off = row_map if row_map is not None else (max(M, 1), 0, 0)
  a, ar = _a(x2d)
  wd = decode_weight(w) if M <= 32 else None
  if wd is not None:
    ops.gemm_linear_(a, wd, bias, resid, out, act, div, mul, off, True, ar)
  else:
    ops.gemm_linear_(a, w, bias, resid, out, act, div, mul, off, False, ar)
  return out


def qkv_rope_decode(x2d, w_perm, positions, H, hd):
  """Decode q, k, v (RoPE applied) from the permuted q|k|v weight."""
  a, ar, wd, nm = _an(x2d, w_perm)
  table = rope_table(w_perm.device, hd)
  ne = float(nm.eps) if nm is not None else 0.0
  if wd is not None:
    return ops.qkv_rope_decode(a, wd, positions, H, hd, table, True, ar,
                               nm is not None, ne)
  return ops.qkv_rope_decode(a, w_perm, positions, H, hd, table, False, ar)


def linear_conv1d_(x2d, w, bias, conv_w, conv_b, conv_state):
  """Decode recurrent-block input projection: (y, conv1d_step(x)) as one
  [M, 2E] tensor, the conv state advanced in place."""
  a, ar, wd, nm = _an(x2d, w)
  if wd is not None:
    return ops.gemm_linear_conv1d_(a, wd, bias, conv_w, conv_b, conv_state, True, ar,
                                   nm is not None,
                                   float(nm.eps) if nm is not None else 0.0)
  return ops.gemm_linear_conv1d_(a, w, bias, conv_w, conv_b, conv_state, False, ar)


FRONT_ONE_LAUNCH = False  # True: the one-launch front where it fits (A/B: tools/front_ab.py)


def recurrent_decode_front_(x2d, w, bias, conv_w, conv_b, conv_state, gates, pos_flat, h):
  """The decode recurrent-block front (y|x projection + Conv1D step + RG-LRU
  gates + scan step, gate = y) as one launch when the rows and shapes fit
  its plan: PackedRows y, conv_state / h advanced in place.  None otherwise
  (the caller runs linear_conv1d_ + rglru_step_)."""
  if not FRONT_ONE_LAUNCH:
    return None
  M, E = x2d.shape[0], conv_w.shape[1]
  wgt, bx, ba, sp = gates
  H, _, bw = wgt.shape
  if not (isinstance(x2d, PackedRows) and x2d.data.is_cuda and conv_w.shape[0] == 4 and
          _lib.load().cadence_recurrent_decode_front_plan(M, E, w.shape[1], H, bw)):
    return None
  wg = decode_weight(wgt)
  if wg is None:
    return None
  a, ar, wd, nm = _an(x2d, w)
  if wd is None:
    return None
  cnt, err = _counters(x2d.device, 64 * H), wait_err(x2d.device)
  if cnt is None or err is None:
    return None
  _, y = ops.recurrent_decode_front(a, ar, wd, bias, conv_w, conv_b, conv_state, wg, bx, ba,
                                    sp, pos_flat, h, cnt, err, nm is not None,
                                    float(nm.eps) if nm is not None else 0.0)
  return PackedRows(y, M, E)


def linear_rmsnorm(x2d, w, bias, resid, norm, packed_out=None, lazy=False):
  """(x2d . w^T + bias + resid, norm(that)) for a layers.RMSNorm `norm`; the
  norm output is PackedRows for decode rows (it only feeds GEMMs).

  lazy (decode rows whose consumer is a norm-aware GEMV): one launch, the
  norm left to the consumer -- PackedRows of the unnormalised rows with
  `norm` set (cadence_gemm_linear_residual_rows)."""
  M, N = x2d.shape[0], w.shape[0]
  if packed_out is None:
    packed_out = want_packed(M, N)
  a, ar = _a(x2d)
  wd = decode_weight(w) if M <= 32 else None
  K = w.shape[1]
  if (lazy and packed_out and wd is not None and resid is not None and
      N % 64 == 0 and N <= 2560 and
      _lib.load().cadence_gemm_rmsnorm_workspace_bytes(M, N, K) > 0 and
      _counters(x2d.device, N // 16) is not None):
    out, rows = ops.gemm_linear_residual_rows(a, wd, bias, resid, True, ar)
    return out, PackedRows(rows, M, N, norm, out)
  out, nout = ops.gemm_linear_rmsnorm(a, wd if wd is not None else w, bias, resid,
                                      norm.scale, norm.eps, wd is not None, ar,
                                      packed_out)
  return out, (PackedRows(nout, M, N) if packed_out else nout)


def gated_gelu(x2d, w_packed, bias_gate, bias_up, packed_out=None):
  """MLP up + gate (packed [2F, K] weight); decode rows use its packed copy
  and emit PackedRows (the output only feeds ffw_down)."""
  M, F = x2d.shape[0], w_packed.shape[0] // 2
  if packed_out is None:
    packed_out = want_packed(M, F)
  a, ar, wd, nm = _an(x2d, w_packed)
  out = ops.gated_gelu(a, wd if wd is not None else w_packed, bias_gate, bias_up,
                       wd is not None, ar, packed_out, nm is not None,
                       float(nm.eps) if nm is not None else 0.0)
  return PackedRows(out, M, F) if packed_out else out


def rglru_gates(x2d, w_packed, bias_x, bias_a, softplus_a, pos_flat):
  wd = decode_weight(w_packed) if x2d.shape[0] <= 32 else None
  if wd is not None:
    return ops.rglru_gates(x2d, wd, bias_x, bias_a, softplus_a, pos_flat, True)
  return ops.rglru_gates(x2d, w_packed, bias_x, bias_a, softplus_a, pos_flat)


def rglru_step_(x2d, w_packed, bias_x, bias_a, softplus_a, pos_flat, h, gate,
                packed_out=None):
  """Gate GEMM + chain + scan step; y is PackedRows for decode rows (it only
  feeds linear_out)."""
  M, E = x2d.shape
  if packed_out is None:
    packed_out = want_packed(M, E)
  wd = decode_weight(w_packed) if M <= 32 else None
  y = ops.rglru_step_(x2d, wd if wd is not None else w_packed, bias_x, bias_a,
                      softplus_a, pos_flat, h, gate, wd is not None, packed_out)
  return PackedRows(y, M, E) if packed_out else y


def logits_argmax(x2d, embedding, soft_cap, return_logits):
  a, ar = _a(x2d)
  wd = decode_weight(embedding) if x2d.shape[0] <= 32 else None
  if wd is not None:
    return ops.logits_argmax(a, wd, soft_cap, return_logits, True, ar)
  return ops.logits_argmax(a, embedding, soft_cap, return_logits, False, ar)


def logits_argmax_tail(x2d, embedding, soft_cap, tail: dict):
  """logits_argmax + decode_advance_ + embed_packed_ of the next token in one
  tail launch (tail: the decode_advance_ operands and the next step's rows,
  see Griffin.next_token_chained)."""
  a, ar = _a(x2d)
  wd = decode_weight(embedding) if x2d.shape[0] <= 32 else None
  w, lay = (wd, True) if wd is not None else (embedding, False)
  return ops.logits_argmax_tail_(
      a, w, soft_cap, lay, ar, tail["buf"], tail["step"], tail["pos"], tail["cur"],
      tail["done"], *tail["eos_args"], tail["counter"], embedding, tail["scale"],
      tail["x"], tail["xp"])


def gemm_logits(x2d, embedding, soft_cap):
  a, ar = _a(x2d)
  wd = decode_weight(embedding) if x2d.shape[0] <= 32 else None
  if wd is not None:
    return ops.gemm_logits(a, wd, soft_cap, True, ar)
  return ops.gemm_logits(a, embedding, soft_cap, False, ar)


def rmsnorm(x2d, scale, eps=1e-6, packed: bool = False):
  """RMSNorm rows; packed=True (only for a GEMM consumer) returns PackedRows
  when the rows qualify (want_packed)."""
  if packed and want_packed(x2d.shape[0], x2d.shape[1]):
    return PackedRows(ops.rmsnorm(x2d, scale, eps, True), x2d.shape[0],
                      x2d.shape[1])
  return ops.rmsnorm(x2d, scale, eps)


def local_attention_decode_(q, k, v, cache_k, cache_v, num_tokens, H):
  """Decode attention step; the output is PackedRows for decode rows (it
  only feeds proj_final)."""
  B = q.shape[0]
  hd = k.shape[-1]
  pk = want_packed(B, H * hd)
  out = ops.local_attention_decode_(q, k, v, cache_k, cache_v, num_tokens, H, pk)
  return PackedRows(out, B, H * hd) if pk else out
