"""Per-kernel parity: gfx950 ops vs the CPU oracle (oracle/griffin_ref.py).

Bit-exact where the kernel reproduces the reference op order (scan, conv,
embedding, RoPE); tolerance-based where only the fp32 accumulation order of
a reduction differs (GEMM, RMSNorm mean, attention, gate chain fed by a
GEMM).  Tolerances follow the reference's own bf16 cross-check
(`recurrentgemma/torch/layers_test.py:131,170`: rtol 1e-2, atol 3e-2).
"""

import math

import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close_bf16, cosine, rel_l2
from oracle import griffin_ref as R

import cadence
from cadence import ops

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, scale=1.0, dtype=BF, gen=None):
  return (torch.randn(*shape, generator=gen) * scale).to(dtype)


def two_doc_positions(b, t, split):
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  pos[:, split:] = torch.arange(t - split, dtype=torch.int32)
  return pos


# ------------------------------------------------------------------ scan

def _chunked(b, t, e):
  """True when cadence_rnn_scan takes the time-chunked form for this shape."""
  from cadence import _lib
  return _lib.load().cadence_rnn_scan_workspace_bytes(b, t, e) > 0


def assert_scan(y, y_ref, h, h_ref, b, t, e):
  """Bit-exact for the sequential kernel; for the chunked form (small
  batches) the first two chunks (>= 16 steps) are bit-exact and later
  chunks differ only through the carry's rounding: >= 99.5 % of y
  bit-equal, within one bf16 ulp elsewhere, fp32 h_last to rtol 1e-4."""
  y, h = y.cpu().view(y_ref.shape), h.cpu()
  if not _chunked(b, t, e):
    assert torch.equal(y, y_ref)
    assert torch.equal(h, h_ref)
    return
  y, y_ref = y.view(b, t, e), y_ref.view(b, t, e)
  assert torch.equal(y[:, :16], y_ref[:, :16])
  frac = (y == y_ref).float().mean().item()
  assert frac >= 0.995, frac
  torch.testing.assert_close(y.float(), y_ref.float(), rtol=8e-3, atol=1e-5)
  torch.testing.assert_close(h, h_ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("b,t,e,with_h0", [(2, 32, 128, True), (3, 129, 256, False),
                                           (1, 1, 64, True), (4, 320, 2560, True),
                                           (1, 319, 2560, False),
                                           (1, 2048, 2560, True),
                                           (26, 64, 2560, True)])
def test_rnn_scan_bitexact(dev, b, t, e, with_h0):
  g = torch.Generator().manual_seed(0)
  x = rnd(b, t, e, gen=g)
  a = torch.rand(b, t, e, generator=g).to(BF)
  reset = torch.rand(b, t, generator=g) < 0.05
  reset[:, 0] = True
  h0 = torch.randn(b, e, generator=g) if with_h0 else None
  y_ref, h_ref = R.rnn_scan(x, a, reset, h0)
  y, h = cadence.rnn_scan(x.to(dev), a.to(dev), reset.to(dev),
                          None if h0 is None else h0.to(dev))
  assert_scan(y, y_ref, h, h_ref, b, t, e)


def test_rnn_scan_chunked_long_decay(dev):
  """Chunked scan with a close to 1 (slow decay: carry errors persist
  longest) and no resets, B = 1, T = 2048: still within the chunk bar."""
  g = torch.Generator().manual_seed(7)
  b, t, e = 1, 2048, 1280
  assert _chunked(b, t, e)
  x = rnd(b, t, e, gen=g)
  a = (0.999 - 0.01 * torch.rand(b, t, e, generator=g)).to(BF)
  reset = torch.zeros(b, t, dtype=torch.bool)
  y_ref, h_ref = R.rnn_scan(x, a, reset, None)
  y, h = cadence.rnn_scan(x.to(dev), a.to(dev), reset.to(dev), None)
  assert_scan(y, y_ref, h, h_ref, b, t, e)
  # in place form (h0 and h_last alias) continues the same state
  hh = torch.zeros(b, e, device=dev)
  y2 = ops.ops.rnn_scan_(x.view(-1, e).to(dev), a.view(-1, e).to(dev), hh,
                         None, b, t)
  assert torch.equal(y2.view(b, t, e).cpu(), y.cpu())
  assert torch.equal(hh.cpu(), h.cpu())


@pytest.mark.parametrize("t,e,strided,with_h0", [(70, 512, False, False),
                                                 (300, 2560, True, True),
                                                 (2048, 256, True, False),
                                                 (33, 192, True, True)])
def test_rnn_scan_gated_matches_join(dev, t, e, strided, with_h0):
  """scan(x, a) * gate fused == reference rnn_scan then `x * y`; the gate may
  be the y half of the packed [y | x] GEMM output (row stride 2E)."""
  g = torch.Generator().manual_seed(1)
  b = 2
  x = rnd(b, t, e, gen=g)
  yx = rnd(b * t, 2 * e, gen=g)
  gate = yx[:, :e] if strided else yx[:, :e].contiguous()
  a = torch.rand(b, t, e, generator=g).to(BF)
  pos = two_doc_positions(b, t, t // 2 + 1)
  h0 = torch.randn(b, e, generator=g) if with_h0 else None
  y_ref, h_ref = R.rnn_scan(x, a, pos == 0, h0)
  want = y_ref * gate.reshape(b, t, e)
  gate_d = yx.to(dev)[:, :e] if strided else gate.to(dev)
  got, h = ops.ops.rnn_scan(x.view(-1, e).to(dev), a.view(-1, e).to(dev),
                            pos.to(dev), None if h0 is None else h0.to(dev),
                            gate_d, b, t)
  assert_scan(got, want, h, h_ref, b, t, e)


# ---------------------------------------------------------------- conv1d

@pytest.mark.parametrize("compat", [True, False])
@pytest.mark.parametrize("b,t,e", [(2, 40, 128), (1, 2, 64), (3, 97, 2560),
                                   (2, 4, 64), (2, 5, 64), (3, 7, 128), (4, 319, 2560)])
def test_conv1d_prefill_bitexact(dev, compat, b, t, e):
  """Conv1D prefill vs the oracle, bitwise: L < 4 (one-step kernel), L >= 4
  (four time steps per thread: ragged last groups, document starts inside
  a group, the bench's 319-step rows)."""
  g = torch.Generator().manual_seed(2)
  x = rnd(b, t, e, gen=g)
  w = rnd(4, e, scale=0.5, gen=g)
  bias = rnd(e, scale=0.1, gen=g)
  pos = two_doc_positions(b, t, max(1, t // 3))
  y_ref, c_ref = R.conv1d(x, pos, w, bias, None, compat=compat)
  conv = cadence.Conv1D(e, 4, device=dev, dtype=BF, compat=compat)
  with torch.no_grad():
    conv.w.copy_(w)
    conv.b.copy_(bias)
  y, c = conv(x.to(dev), pos.to(dev))
  assert torch.equal(y.cpu(), y_ref)
  assert torch.equal(c.cpu(), c_ref)


def test_conv1d_decode_bitexact(dev):
  g = torch.Generator().manual_seed(3)
  b, e = 4, 256
  x = rnd(b, 1, e, gen=g)
  cache = rnd(b, 3, e, gen=g)
  w, bias = rnd(4, e, gen=g), rnd(e, gen=g)
  pos = torch.full((b, 1), 7, dtype=torch.int32)
  y_ref, c_ref = R.conv1d(x, pos, w, bias, cache)
  conv = cadence.Conv1D(e, 4, device=dev, dtype=BF)
  with torch.no_grad():
    conv.w.copy_(w)
    conv.b.copy_(bias)
  y, c = conv(x.to(dev), pos.to(dev), cache.to(dev))
  assert torch.equal(y.cpu(), y_ref)
  assert torch.equal(c.cpu(), c_ref)


# --------------------------------------------------------------- RMSNorm

@pytest.mark.parametrize("rows,width", [(5, 128), (300, 2560), (1, 1024)])
def test_rmsnorm(dev, rows, width):
  g = torch.Generator().manual_seed(4)
  x = rnd(rows, width, scale=3.0, gen=g)
  scale = rnd(width, scale=0.2, gen=g)
  want = R.rms_norm(x, scale)
  norm = cadence.RMSNorm(width, device=dev, dtype=BF)
  with torch.no_grad():
    norm.scale.copy_(scale)
  got = norm(x.to(dev))
  # torch's CPU bf16 rsqrt is an approximation (not correctly rounded), so
  # a row's scale can differ by one bf16 ulp: tolerance, not bit-equality.
  assert_close_bf16(got, want, rtol=2e-2, atol=2e-2, what="rmsnorm")
  assert cosine(got, want) > 0.9999


def test_rmsnorm_kat(dev):
  """recurrentgemma/jax/layers_test.py:63-69 (zero scale)."""
  x = torch.tensor([[0.1, 0.2]], dtype=torch.float32)
  want = torch.tensor([[0.6324429, 1.2648858]])
  norm = cadence.RMSNorm(8, device=dev, dtype=BF)   # width must be % 8
  xx = torch.zeros(1, 8)
  xx[0, :2] = x
  got = norm(xx.to(BF).to(dev)).float().cpu()
  ref = R.rms_norm(xx.to(BF), torch.zeros(8, dtype=BF)).float()
  torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)
  # the KAT itself is a width-2 row: check the bf16 oracle reproduces it
  k = R.rms_norm(x.to(BF), torch.zeros(2, dtype=BF)).float()
  torch.testing.assert_close(k, want, rtol=1e-2, atol=1e-2)


# ------------------------------------------------------------------ GEMMs

@pytest.mark.parametrize("m,n,k", [(1, 128, 64), (17, 256, 256), (64, 2560, 2560),
                                   (65, 128, 128), (300, 384, 640),
                                   (1000, 5120, 2560)])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_linear(dev, m, n, k, act):
  g = torch.Generator().manual_seed(5)
  a = rnd(m, k, gen=g)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g)
  bias = rnd(n, scale=0.1, gen=g)
  want = F.linear(a.float(), w.float(), bias.float())
  if act == 1:
    want = F.gelu(want.to(BF).float())
  got = ops.linear(a.to(dev), w.to(dev), bias.to(dev), act=act)
  assert_close_bf16(got, want.to(BF), rtol=1e-2, atol=1e-2, what="linear")


@pytest.mark.parametrize("m,n,k", [(32, 2560, 2560), (32, 2560, 7680),
                                   (5, 192, 96), (17, 4096, 2560)])
def test_decode_packed_layout_bitwise(dev, m, n, k):
  """The fragment-packed decode copy (ldw == 0) gives bit-identical results to
  the row-major weight: same engine, same summation order."""
  g = torch.Generator().manual_seed(11)
  a = rnd(m, k, gen=g).to(dev)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g).to(dev)
  bias = rnd(n, scale=0.1, gen=g).to(dev)
  resid = rnd(m, n, gen=g).to(dev)
  wp = ops.pack_decode(w)
  o1 = torch.empty(m, n, dtype=BF, device=dev)
  o2 = torch.empty(m, n, dtype=BF, device=dev)
  ops.ops.gemm_linear_(a, w, bias, resid, o1, 0, m, 0, 0)
  ops.ops.gemm_linear_(a, wp, bias, resid, o2, 0, m, 0, 0, True)
  assert torch.equal(o1, o2)
  assert torch.equal(ops.linear(a, w, bias, resid=resid), o1)   # auto-packed
  if n % 128 == 0:       # gated kernel contract: F % 64 == 0
    f = n // 2
    bg, bu = rnd(f, scale=0.1, gen=g).to(dev), rnd(f, scale=0.1, gen=g).to(dev)
    g1 = ops.ops.gated_gelu(a, w, bg, bu)
    g2 = ops.ops.gated_gelu(a, wp, bg, bu, True)
    assert torch.equal(g1, g2)
  lg1, n1 = ops.ops.logits_argmax(a, w, 30.0, True)
  lg2, n2 = ops.ops.logits_argmax(a, wp, 30.0, True, True)
  assert torch.equal(lg1, lg2) and torch.equal(n1, n2)


def test_decode_packed_rglru_gates_bitwise(dev):
  g = torch.Generator().manual_seed(12)
  h, bw, m = 10, 256, 32
  x = rnd(m, h * bw, gen=g).to(dev)
  w = rnd(h, 2 * bw, bw, scale=1 / 16, gen=g).to(dev)
  bx, ba = rnd(h * bw, scale=0.3, gen=g).to(dev), rnd(h * bw, scale=0.3, gen=g).to(dev)
  sp = torch.rand(h * bw, generator=g).to(BF).to(dev)
  pos = torch.randint(0, 3, (m,), generator=g, dtype=torch.int32).to(dev)
  a1, x1 = ops.ops.rglru_gates(x, w, bx, ba, sp, pos)
  a2, x2 = ops.ops.rglru_gates(x, ops.pack_decode(w), bx, ba, sp, pos, True)
  assert torch.equal(a1, a2) and torch.equal(x1, x2)


@pytest.mark.parametrize("m,h,bw", [(10208, 10, 256), (319, 10, 256), (33, 10, 256),
                                    (100, 4, 128), (77, 2, 64), (4096, 8, 128)])
def test_prefill_rglru_gates_stream_kernel_bitwise(dev, m, h, bw):
  """The prefill gates kernel (rglru_gates_stream_kernel: block-bound
  workgroups, weights in registers, 32-row tiles) against the block engine
  it replaced (lab switch engine 0), bitwise: same MFMA k order, same
  chain.  Resets, a ragged last tile, every block width it takes, and the
  bench shape (32 x 319 rows)."""
  from cadence import _lib
  g = torch.Generator().manual_seed(31)
  e = h * bw
  x = rnd(m, 2 * e, gen=g).to(dev)[:, e:]          # strided: the y|x GEMM output
  w = rnd(h, 2 * bw, bw, scale=1 / math.sqrt(bw), gen=g).to(dev)
  bx, ba = rnd(e, scale=0.3, gen=g).to(dev), rnd(e, scale=0.3, gen=g).to(dev)
  sp = torch.rand(e, generator=g).to(BF).to(dev)
  pos = torch.randint(0, 5, (m,), generator=g, dtype=torch.int32).to(dev)
  lib = _lib.load()
  a1, x1 = ops.ops.rglru_gates(x, w, bx, ba, sp, pos)
  prev = lib.cadence_gemm_set_engine(0)
  try:
    a0, x0 = ops.ops.rglru_gates(x, w, bx, ba, sp, pos)
  finally:
    lib.cadence_gemm_set_engine(prev)
  if m > 64 and lib.cadence_gemm_big_splits(m, 2 * bw, bw, h) == 1:
    assert torch.equal(a1, a0) and torch.equal(x1, x0)
  else:
    # for this small M the old path split K (the skinny engine's wave
    # partials at M <= 64, or split-K partials) and summed in another
    # order: the unsplit chain rounds a few sums differently
    assert_close_bf16(a1, a0, rtol=1e-2, atol=1e-2, min_equal=0.99, what="a")
    assert_close_bf16(x1, x0, rtol=1e-2, atol=1e-2, min_equal=0.99, what="nx")
  assert bool((a1[pos == 0] == 0).all())


@pytest.mark.parametrize("packed", [False, True])
def test_rglru_step_matches_gates_then_scan(dev, packed):
  """Fused decode step == gate chain then rnn_scan's T == 1 branch, bitwise,
  with resets, a non-zero state and the y gate (row stride 2E)."""
  g = torch.Generator().manual_seed(13)
  h_, bw, m = 10, 256, 32
  e = h_ * bw
  x = rnd(m, e, gen=g).to(dev)
  yx = rnd(m, 2 * e, gen=g).to(dev)
  gate = yx[:, :e]
  w = rnd(h_, 2 * bw, bw, scale=1 / 16, gen=g).to(dev)
  bx, ba = rnd(e, scale=0.3, gen=g).to(dev), rnd(e, scale=0.3, gen=g).to(dev)
  sp = torch.rand(e, generator=g).to(BF).to(dev)
  pos = torch.randint(0, 3, (m,), generator=g, dtype=torch.int32).to(dev)
  h0 = torch.randn(m, e, generator=g).to(dev)
  a, nx = ops.ops.rglru_gates(x, w, bx, ba, sp, pos)
  h_ref = h0.clone()
  want = ops.ops.rnn_scan_(nx, a, h_ref, gate, m, 1)
  h = h0.clone()
  wk = ops.pack_decode(w) if packed else w
  got = ops.ops.rglru_step_(x, wk, bx, ba, sp, pos, h, gate, packed)
  assert torch.equal(got, want)
  assert torch.equal(h, h_ref)


@pytest.mark.parametrize("m,n,k", [(32, 2560, 2560), (32, 2560, 7680),
                                   (16, 2560, 7680), (5, 2560, 2560),
                                   (24, 1024, 2560), (8, 4096, 10240),
                                   (7, 512, 256), (100, 512, 256)])
def test_gemm_linear_rmsnorm(dev, m, n, k):
  """Residual GEMM fused with the following RMSNorm (decode: split-K finished
  by the row-owned reduce+norm kernel; M <= 16, N too narrow for two column
  tiles per block, 4 splits) vs linear then rmsnorm."""
  g = torch.Generator().manual_seed(14)
  a = rnd(m, k, gen=g).to(dev)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g).to(dev)
  bias = rnd(n, scale=0.1, gen=g).to(dev)
  resid = rnd(m, n, gen=g).to(dev)
  norm = cadence.layers.RMSNorm(n, device=dev, dtype=BF)
  with torch.no_grad():
    norm.scale.copy_(rnd(n, scale=0.2, gen=g))
  out, nout = ops.linear_rmsnorm(a, w, bias, resid, norm)
  if isinstance(nout, ops.PackedRows):     # decode rows: packed norm output
    nout = nout.unpack()
  ref = ops.linear(a, w, bias, resid=resid)
  if m > 64:   # prefill: the same two kernels
    assert torch.equal(out, ref)
    assert torch.equal(nout, ops.rmsnorm(ref, norm.scale, norm.eps))
  else:        # split-K order differs: bf16 tolerance
    assert_close_bf16(out, ref.cpu(), rtol=1e-2, atol=2e-2, what="resid gemm")
    want = R.rms_norm(out.cpu(), norm.scale.cpu())
    assert_close_bf16(nout, want, rtol=2e-2, atol=2e-2, what="fused norm")


def test_gemm_linear_residual_rowmap(dev):
  g = torch.Generator().manual_seed(6)
  m, n, k = 96, 256, 128
  a = rnd(m, k, gen=g)
  w = rnd(n, k, scale=0.1, gen=g)
  # rows of 12 scattered into 20-row groups at offset 5
  out = torch.zeros(8 * 20, n, dtype=BF, device=dev)
  ops.linear(a.to(dev), w.to(dev), out=out, row_map=(12, 20, 5))
  want = F.linear(a.float(), w.float()).to(BF).view(8, 12, n)
  got = out.view(8, 20, n).cpu()
  assert_close_bf16(got[:, 5:17], want, rtol=1e-2, atol=1e-2)
  assert torch.all(got[:, :5] == 0) and torch.all(got[:, 17:] == 0)
  resid = rnd(m, n, gen=g)
  got = ops.linear(a.to(dev), w.to(dev), resid=resid.to(dev))
  want = (F.linear(a.float(), w.float()).to(BF) + resid)
  assert_close_bf16(got, want, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("m", [8, 200])
def test_gated_gelu(dev, m):
  g = torch.Generator().manual_seed(7)
  d, f = 256, 768
  x = rnd(1, m, d, gen=g)
  mlp = cadence.MLPBlock(d, f, device=dev, dtype=BF)
  with torch.no_grad():
    mlp.ffw_up.w.copy_(rnd(2, d, f, scale=1 / 16, gen=g))
    mlp.ffw_up.b.copy_(rnd(2, 1, 1, f, scale=0.1, gen=g))
  p = {k: v.cpu() for k, v in mlp.state_dict().items()}
  want = R.mlp_block(x, p, "")
  got = mlp(x.to(dev))
  assert_close_bf16(got, want, rtol=2e-2, atol=2e-2, what="mlp")
  assert cosine(got, want) > 0.9999


@pytest.mark.parametrize("m", [16, 150])
def test_rglru_block_vs_oracle(dev, m):
  g = torch.Generator().manual_seed(8)
  e, h = 512, 2
  b, t = 2, m // 2
  x = rnd(b, t, e, gen=g)
  pos = two_doc_positions(b, t, t // 3)
  lru = cadence.RGLRU(e, h, device=dev, dtype=BF)
  with torch.no_grad():
    lru.input_gate.b.copy_(rnd(h, e // h, scale=0.5, gen=g))
    lru.a_gate.b.copy_(rnd(h, e // h, scale=0.5, gen=g))
  p = {k: v.cpu() for k, v in lru.state_dict().items()}
  h0 = torch.randn(b, e, generator=g)
  y_ref, h_ref = R.rg_lru(x, pos, p, "", h0)
  y, hl = lru(x.to(dev), pos.to(dev), h0.to(dev))
  assert_close_bf16(y, y_ref, rtol=2e-2, atol=2e-2, min_equal=0.9, what="rglru")
  torch.testing.assert_close(hl.cpu(), h_ref, rtol=2e-2, atol=2e-2)


# ------------------------------------------------------------- attention

def _attn_ref(q, k, v, pos, window):
  """Oracle attention from already-rotated q [B,T,H,hd], k/v [B,T,hd]."""
  hd = q.shape[-1]
  mask = R.prefill_mask(pos, window)
  logits = torch.einsum("btnh,bsh->bnts", q, k) * (hd ** -0.5)
  logits = torch.where(mask[:, None], logits, R.MIN_LOGIT).float()
  probs = torch.softmax(logits, -1).to(BF)
  return torch.einsum("bnts,bsh->btnh", probs, v)


@pytest.mark.parametrize("b,t,h,hd,window,split", [
    (2, 96, 4, 64, 2048, 40), (1, 150, 10, 256, 2048, 100),
    (2, 200, 2, 128, 48, 0), (3, 33, 3, 256, 16, 7)])
def test_rope_and_local_attention(dev, b, t, h, hd, window, split):
  g = torch.Generator().manual_seed(9)
  qkv = rnd(b * t, (h + 2) * hd, gen=g)
  pos = two_doc_positions(b, t, split) if split else \
      torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  q = qkv[:, :h * hd].view(b, t, h, hd)
  k = qkv[:, h * hd:(h + 1) * hd].view(b, t, 1, hd)
  v = qkv[:, (h + 1) * hd:].view(b, t, hd)
  q_ref = R.apply_rope(q, pos)
  k_ref = R.apply_rope(k, pos)[:, :, 0]
  qd, kd, vd = ops.ops.rope_qkv(qkv.to(dev), pos.to(dev).view(-1), h, hd)
  assert_close_bf16(qd.view(b, t, h, hd), q_ref, rtol=1e-2, atol=1e-2,
                    min_equal=0.995, what="rope q")
  assert_close_bf16(kd.view(b, t, hd), k_ref, rtol=1e-2, atol=1e-2,
                    min_equal=0.995, what="rope k")
  assert torch.equal(vd.cpu().view(b, t, hd), v)
  want = _attn_ref(q_ref, k_ref, v, pos, window)
  seg, start = ops.ops.segment_info(pos.to(dev))
  got = ops.ops.local_attention(qd, kd, vd, seg, start, b, t, h, hd, window)
  got = got.view(b, t, h, hd)
  assert_close_bf16(got, want, rtol=3e-2, atol=3e-2, what="local attention")
  assert rel_l2(got, want) < 1e-2


@pytest.mark.parametrize("m,h,hd,k", [(32 * 319, 10, 256, 2560), (32 * 639, 10, 256, 2560),
                                      (8 * 319, 10, 256, 2560)])
def test_qkv_rope_prefill_matches_two_launch_form(dev, m, h, hd, k):
  """Prompt-pass q|k|v GEMM with RoPE in the staged epilogue (permuted
  weight rows) == linear on the natural rows, then rope_qkv: bitwise (same
  per-column MFMA chains, same rotation arithmetic).  Positions include
  document resets, -1 padding and positions past the sin / cos table."""
  assert ops.qkv_rope_prefill_ok(m, h, hd, k), "plan should be one unsplit launch"
  g = torch.Generator().manual_seed(21)
  x = rnd(m, k, gen=g).to(dev)
  w = rnd((h + 2) * hd, k, scale=1 / math.sqrt(k), gen=g).to(dev)
  pos = torch.randint(-1, 3000, (m,), generator=g, dtype=torch.int32)
  pos[::7] = 0
  pos[5] = ops.ROPE_TABLE_POSITIONS + 17
  pos = pos.to(dev)
  table = ops.rope_table(dev, hd)
  qkv = ops.linear(x, w)
  q0, k0, v0 = ops.ops.rope_qkv(qkv, pos, h, hd, table)
  wp = w[ops.qkv_rope_permutation(h, hd, dev)].contiguous()
  q1, k1, v1 = ops.ops.qkv_rope_prefill(x, wp, pos, h, hd, table)
  assert torch.equal(v1, v0)
  assert torch.equal(k1, k0)
  assert torch.equal(q1, q0)


@pytest.mark.parametrize("m,h,hd,k", [(319, 10, 256, 2560), (300, 4, 128, 512),
                                      (1000, 6, 64, 512)])
def test_qkv_split_k_then_rope_path(dev, m, h, hd, k):
  """The q|k|v path of shapes the fused prefill launch does not cover (C3's
  B = 1 prompt, M = 319: split-K partial GEMM + reduce, then rope_qkv).
  The attention block's forward equals the explicit two-launch composition
  bitwise (so it takes this path and nothing else); the split-K GEMM is
  within one bf16 rounding of an fp32 matmul (>= 98 % bit-equal), and the
  rotation of its output matches the oracle's RoPE on the same rows
  (>= 99.5 % bit-equal: sin / cos rounding)."""
  from cadence import _lib
  n = (h + 2) * hd
  lib = _lib.load()
  assert not ops.qkv_rope_prefill_ok(m, h, hd, k)
  g = torch.Generator().manual_seed(22)
  x = rnd(m, k, gen=g)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g)
  pos = torch.randint(-1, 3000, (m,), generator=g, dtype=torch.int32)
  pos[::7] = 0
  xd, wd, pd = x.to(dev), w.to(dev), pos.to(dev)
  qkv = ops.linear(xd, wd)
  want = (x.float() @ w.float().t()).to(BF)
  assert_close_bf16(qkv, want, rtol=1e-2, atol=1e-2, min_equal=0.98, what="split-K qkv")
  table = ops.rope_table(dev, hd)
  q, kk, v = ops.ops.rope_qkv(qkv, pd, h, hd, table)
  assert torch.equal(v.cpu(), qkv.cpu()[:, (h + 1) * hd:])
  qc = qkv.cpu()
  q_ref = R.apply_rope(qc[:, :h * hd].view(1, m, h, hd), pos[None]).view(m, h * hd)
  k_ref = R.apply_rope(qc[:, h * hd:(h + 1) * hd].view(1, m, 1, hd), pos[None]).view(m, hd)
  assert_close_bf16(q, q_ref, rtol=1e-2, atol=1e-2, min_equal=0.995, what="rope q")
  assert_close_bf16(kk, k_ref, rtol=1e-2, atol=1e-2, min_equal=0.995, what="rope k")
  if h * hd > 2560 or hd != 256:
    return
  # the block's own forward at this shape (B = 1, T = m) == the composition
  blk = cadence.LocalAttentionBlock(h * hd, h, window_size=2048, device=dev, dtype=BF)
  with torch.no_grad():
    blk.proj_q.weight.copy_(w[:h * hd])
    blk.proj_k.weight.copy_(w[h * hd:(h + 1) * hd])
    blk.proj_v.weight.copy_(w[(h + 1) * hd:])
  p2 = torch.arange(m, dtype=torch.int32)[None].to(dev)
  got, _ = blk(xd[None], p2, return_cache=False)
  q, kk, v = ops.ops.rope_qkv(qkv, p2.view(-1), h, hd, table)
  seg, start = ops.ops.segment_info(p2)
  enc = ops.ops.local_attention(q, kk, v, seg, start, 1, m, h, hd, 2048)
  ref = ops.linear(enc, blk.proj_final.weight, blk.proj_final.bias,
                   resid=torch.zeros(m, h * hd, dtype=BF, device=dev))
  assert torch.equal(got.view(m, -1), ref)


@pytest.mark.parametrize("b,ctx", [(32, 352), (1, 1500), (2, 2100), (4, 0)])
def test_decode_attention_ranges(dev, b, ctx):
  """Decode attention at the bench batch (8 key ranges per sequence, one
  tile each), a single sequence (32 ranges: the combine's second group), a
  wrapped 2048-slot ring (several 64-key tiles per range) and an empty
  cache (only the new key), against the reference's cache mask
  (modules.py:155-185) and ring update (modules.py:206-218)."""
  g = torch.Generator().manual_seed(20 + b)
  h, hd, window = 10, 256, 2048
  ck = rnd(b, window, 1, hd, gen=g)
  cv = rnd(b, window, 1, hd, gen=g)
  nt = torch.tensor([ctx + 3 * i for i in range(b)], dtype=torch.int32)
  q = rnd(b, 1, h, hd, gen=g)
  kn = rnd(b, 1, 1, hd, gen=g)
  vn = rnd(b, 1, 1, hd, gen=g)
  allk = torch.cat([ck, kn], 1)
  allv = torch.cat([cv, vn], 1)
  mask = R.cache_mask(1, nt, window)
  lg = torch.einsum("btnh,bsh->bnts", q, allk[:, :, 0]) * hd ** -0.5
  lg = torch.where(mask[:, None], lg, R.MIN_LOGIT).float()
  want = torch.einsum("bnts,bsh->btnh", torch.softmax(lg, -1).to(BF), allv[:, :, 0])
  ckd, cvd, ntd = ck.view(b, window, hd).to(dev), cv.view(b, window, hd).to(dev), nt.to(dev)
  got = ops.ops.local_attention_decode_(q.to(dev).view(b, h * hd), kn.to(dev).view(b, hd),
                                        vn.to(dev).view(b, hd), ckd, cvd, ntd, h)
  assert_close_bf16(got.view(b, 1, h, hd), want, rtol=3e-2, atol=3e-2,
                    what=f"decode attention b={b} ctx={ctx}")
  assert rel_l2(got.view(b, 1, h, hd), want) < 1e-2
  ckr, cvr = ck.view(b, window, hd).clone(), cv.view(b, window, hd).clone()
  for i in range(b):
    ckr[i, int(nt[i]) % window] = kn[i, 0, 0]
    cvr[i, int(nt[i]) % window] = vn[i, 0, 0]
  assert torch.equal(ckd.cpu(), ckr) and torch.equal(cvd.cpu(), cvr)
  assert torch.equal(ntd.cpu(), nt + 1)
  # replays are bit-identical (fixed combine order)
  again = ops.ops.local_attention_decode_(
      q.to(dev).view(b, h * hd), kn.to(dev).view(b, hd), vn.to(dev).view(b, hd),
      ck.view(b, window, hd).to(dev), cv.view(b, window, hd).to(dev), nt.to(dev), h)
  assert torch.equal(again.cpu(), got.cpu())


def test_kv_cache_fill_and_decode(dev):
  g = torch.Generator().manual_seed(10)
  b, h, hd, window = 3, 4, 256, 64
  for t in (20, 64):
    k = rnd(b, t, hd, gen=g)
    v = rnd(b, t, hd, gen=g)
    pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
    pos[1] = torch.arange(t, dtype=torch.int32) + 37       # wraps the ring
    want = R.cache_from_prompt(k[:, :, None], v[:, :, None], pos, window)
    ck, cv, nt = ops.ops.kv_cache_fill(k.to(dev).view(-1, hd),
                                       v.to(dev).view(-1, hd), pos.to(dev),
                                       window)
    assert torch.equal(ck.cpu(), want["keys"])
    assert torch.equal(cv.cpu(), want["values"])
    assert torch.equal(nt.cpu(), want["num_tokens"])
    # 5 decode steps against the oracle's mask/ring semantics
    ckr, cvr, ntr = want["keys"].clone(), want["values"].clone(), \
        want["num_tokens"].clone()
    for _ in range(5):
      q = rnd(b, 1, h, hd, gen=g)
      kn = rnd(b, 1, 1, hd, gen=g)
      vn = rnd(b, 1, 1, hd, gen=g)
      allk = torch.cat([ckr, kn], 1)
      allv = torch.cat([cvr, vn], 1)
      mask = R.cache_mask(1, ntr, window)
      lg = torch.einsum("btnh,bsh->bnts", q, allk[:, :, 0]) * hd ** -0.5
      lg = torch.where(mask[:, None], lg, R.MIN_LOGIT).float()
      want_o = torch.einsum("bnts,bsh->btnh", torch.softmax(lg, -1).to(BF),
                            allv[:, :, 0])
      for i in range(b):
        s = int(ntr[i]) % window
        ckr[i, s] = kn[i, 0]
        cvr[i, s] = vn[i, 0]
      ntr = ntr + 1
      got = ops.ops.local_attention_decode_(
          q.to(dev).view(b, h * hd), kn.to(dev).view(b, hd),
          vn.to(dev).view(b, hd), ck, cv, nt, h)
      assert_close_bf16(got.view(b, 1, h, hd), want_o, rtol=3e-2, atol=3e-2,
                        what="decode attention")
      assert torch.equal(ck.cpu(), ckr) and torch.equal(cv.cpu(), cvr)
      assert torch.equal(nt.cpu(), ntr.to(torch.int32))


@pytest.mark.parametrize("n,h,hd", [(261, 16, 64), (256, 16, 72), (40, 2, 72),
                                    (581, 16, 64), (576, 16, 72), (734, 16, 64),
                                    (729, 16, 72), (300, 3, 72), (289, 2, 64),
                                    (1, 2, 72), (64, 3, 72), (65, 2, 72), (320, 2, 64),
                                    (385, 1, 64), (129, 5, 72), (40, 2, 64),
                                    (100, 3, 64), (129, 2, 64), (1, 2, 64),
                                    (288, 2, 64)])
def test_vit_attention(dev, n, h, hd):
  """timm SDPA (fp32) vs the LDS-resident kernel (hd 64, N <= 288) and the
  streaming kernel vit_flash_attn_kernel (everything else: SigLIP 224 px,
  the 336 / 384 px towers DINO 581 / 734, SigLIP 576 / 729; tails of 1, 5,
  33 keys and whole tiles; query blocks of 1 to 8 tiles)."""
  g = torch.Generator().manual_seed(11)
  b = 2
  qkv = rnd(b * n, 3 * h * hd, gen=g)
  t = qkv.float().view(b, n, 3, h, hd).permute(2, 0, 3, 1, 4)
  att = torch.softmax((t[0] * hd ** -0.5) @ t[1].transpose(-1, -2), -1)
  want = (att @ t[2]).transpose(1, 2).reshape(b * n, h * hd)
  got = ops.ops.vit_attention(qkv.to(dev), b, n, h, hd)
  assert rel_l2(got, want) < 1e-2
  assert cosine(got, want) > 0.9999


@pytest.mark.parametrize("m,d", [(32 * 261, 1024), (32 * 256, 1152), (7, 1024),
                                 (13, 1152), (4, 64), (5, 1280), (3, 2048)])
def test_layernorm(dev, m, d):
  """The ViT LayerNorm (fp32 residual rows in, bf16 out; timm's eps 1e-6)
  against torch's fp32 layer_norm: the register form (rows up to 1280
  wide) and the looped one beyond, ragged row counts."""
  g = torch.Generator().manual_seed(29)
  x = (torch.randn(m, d, generator=g) * 3 + 0.5).to(dev)
  w = (torch.randn(d, generator=g) * 0.5 + 1).to(torch.bfloat16).to(dev)
  b = (torch.randn(d, generator=g) * 0.2).to(torch.bfloat16).to(dev)
  got = ops.ops.layernorm(x, w, b, 1e-6)
  want = torch.nn.functional.layer_norm(x.cpu(), (d,), w.float().cpu(), b.float().cpu(), 1e-6)
  assert rel_l2(got.float().cpu(), want) < 4e-3


# --------------------------------------------------------------- others

def test_embed_and_logits_argmax(dev):
  g = torch.Generator().manual_seed(12)
  v, d, m = 1024, 256, 7
  emb = rnd(v, d, scale=0.05, gen=g)
  toks = torch.randint(0, v, (m,), generator=g, dtype=torch.int32)
  e = cadence.Embedder(v, d, True, device=dev, dtype=BF)
  with torch.no_grad():
    e.input_embedding.copy_(emb)
  got = e.encode(toks.to(dev))
  cfg = cadence.GriffinConfig(vocab_size=v, width=d, mlp_expanded_width=64,
                              num_heads=4, block_types=(),
                              embeddings_scale_by_sqrt_dim=True,
                              attention_window_size=8, logits_soft_cap=30.0)
  want = R.embed(toks.long(), {"embedder.input_embedding": emb}, cfg)
  assert torch.equal(got.cpu(), want)
  x = rnd(m, d, gen=g)
  lg, nxt = ops.ops.logits_argmax(x.to(dev), e.input_embedding, 30.0, True)
  ref = torch.tanh((x @ emb.T) / 30.0) * 30.0
  assert_close_bf16(lg, ref, rtol=2e-2, atol=3e-2, what="logits")
  # argmax is exact over the kernel's own logits (lowest index on ties)
  assert torch.equal(nxt.cpu().long(), torch.argmax(lg.cpu(), -1))
  full = ops.ops.gemm_logits(x.to(dev), e.input_embedding, 30.0)
  assert torch.equal(full.cpu(), lg.cpu())


def test_library_uses_torch_hip_runtime(dev):
  from cadence import _lib
  _lib.load()
  rts = _lib.hip_runtimes_loaded()
  assert len(rts) == 1, rts


def test_sequence_parallel_scan_chunks_on_gpu(dev):
  """SURVEY 8f f4 carry algebra with the HIP scan, 4 chunks simulated on one
  GPU (the collective is the gloo-tested all-gather), against the ORACLE's
  single-pass scan on the CPU (reference layers.py:145-199): the chunk
  summaries (h_loc, P) equal the oracle's per chunk, and the composed scan
  equals the oracle's one pass up to fp32 rounding of the carry."""
  from cadence import distributed as D
  from oracle import griffin_ref as R
  g = torch.Generator().manual_seed(17)
  b, t, e, chunks = 2, 4096, 2560, 4
  x_c = rnd(b, t, e, gen=g)
  a_c = (0.9 + 0.1 * torch.rand(b, t, e, generator=g)).to(BF)
  reset_c = torch.rand(b, t, generator=g) < 0.001
  h0_c = torch.randn(b, e, generator=g)
  x, a, reset, h0 = x_c.to(dev), a_c.to(dev), reset_c.to(dev), h0_c.to(dev)
  lr = t // chunks
  sls = [slice(i * lr, (i + 1) * lr) for i in range(chunks)]
  stats = torch.stack([D.sp_scan_stats(x[:, s].contiguous(), a[:, s].contiguous(),
                                       reset[:, s].contiguous()) for s in sls])
  stats_ref = torch.stack([D.sp_scan_stats(x_c[:, s], a_c[:, s], reset_c[:, s],
                                           R.rnn_scan) for s in sls])
  # per-chunk summaries: the HIP scan of a chunk (the T-chunked kernel at
  # this batch) against the oracle's sequential one
  torch.testing.assert_close(stats.cpu(), stats_ref, rtol=1e-4, atol=1e-5)
  ys, hs = [], []
  for i, s in enumerate(sls):
    y, h = cadence.rnn_scan(x[:, s].contiguous(), a[:, s].contiguous(),
                            reset[:, s].contiguous(), D.sp_carry_in(stats, i, h0))
    ys.append(y)
    hs.append(h)
  y_ref, h_ref = R.rnn_scan(x_c, a_c, reset_c, h0_c)
  y = torch.cat(ys, 1).cpu()
  # the first steps run from h0 itself in the reference op order: bit-exact;
  # later ones differ only by the fp32 rounding of composed carries
  assert torch.equal(y[:, :16], y_ref[:, :16])
  assert (y == y_ref).float().mean().item() > 0.99
  torch.testing.assert_close(y.float(), y_ref.float(), rtol=1e-2, atol=1e-2)
  torch.testing.assert_close(hs[-1].cpu(), h_ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,l", [(3, 7), (4, 319), (2, 3001)])
def test_segment_info(dev, b, l):
  """seg = cumsum(pos == 0) (modules.py:145) and the start index of each
  row's segment (0 before the first reset), incl. left pads (-1)."""
  g = torch.Generator().manual_seed(b * l)
  pos = torch.randint(1, 50, (b, l), generator=g, dtype=torch.int32)
  pos[torch.rand(b, l, generator=g) < 0.02] = 0
  pos[0, :min(3, l)] = -1                   # left padding, no reset yet
  pos[-1, 0] = 0
  seg, start = ops.ops.segment_info(pos.to(dev))
  want_seg = torch.cumsum((pos == 0).to(torch.int32), 1)
  idx = torch.arange(l)[None].expand(b, l)
  last = torch.where(pos == 0, idx, torch.zeros_like(idx))
  want_start = torch.cummax(last, 1).values
  assert torch.equal(seg.cpu(), want_seg.to(torch.int32))
  assert torch.equal(start.cpu(), want_start.to(torch.int32))


def test_copy_batched_matches_tensor_copies(dev):
  """ops.copy_batched_ (cadence_copy_batched, one launch per 32 regions):
  the decode graph's hand-over copies -- ring-buffer slot prefixes
  [B, :slots], contiguous states, 4-byte int32 vectors, bf16 rows with a
  column offset -- equal Tensor.copy_ bitwise, over more than one batch of
  32 descriptors."""
  g = torch.Generator().manual_seed(31)
  pairs, want = [], []
  for i in range(40):
    b = 1 + i % 3
    if i % 4 == 0:
      src = rnd(b, 64, 1, 32, gen=g).to(dev)
      dst = torch.zeros_like(src)
      s = 1 + i % 50
      pairs.append((dst[:, :s], src[:, :s]))
      w = dst.clone(); w[:, :s] = src[:, :s]; want.append((dst, w))
    elif i % 4 == 1:
      src = torch.randn(b, 96, generator=g).to(dev)
      dst = torch.zeros_like(src)
      pairs.append((dst, src)); want.append((dst, src.clone()))
    elif i % 4 == 2:
      src = torch.randint(0, 1000, (b,), dtype=torch.int32, generator=g).to(dev)
      dst = torch.zeros_like(src)
      pairs.append((dst, src)); want.append((dst, src.clone()))
    else:
      src = torch.randint(0, 1000, (b, 10), dtype=torch.int32, generator=g).to(dev)
      dst = torch.zeros(b, 12, dtype=torch.int32, device=dev)
      pairs.append((dst[:, 3:], src[:, 1:10]))
      w = dst.clone(); w[:, 3:] = src[:, 1:10]; want.append((dst, w))
  ops.copy_batched_(pairs)
  torch.cuda.synchronize()
  for dst, w in want:
    assert torch.equal(dst.cpu(), w.cpu())


@pytest.mark.parametrize("m", [10208, 4500, 300])
def test_gemm_w4_engine_bitwise_vs_8wave(dev, m):
  """The 4-wave prefill engine (gemm_w4_kernel, planned for K >= 2048 and
  N >= 8192) against the 8-wave block engine it replaced (lab switch engine
  0), bitwise: linear, linear + bias + residual (the residual-prefetch
  epilogue, engine bit 2) and the gated-GELU pair epilogue, at the gated
  MLP's N = 15360, K = 2560, with ragged 224 / 256-row tails."""
  from cadence import _lib
  lib = _lib.load()
  n, k = 15360, 2560
  g = torch.Generator().manual_seed(23)
  a = rnd(m, k, gen=g).to(dev)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g).to(dev)
  bias = rnd(n, scale=0.1, gen=g).to(dev)
  resid = rnd(m, n, gen=g).to(dev)
  bg, bu = rnd(n // 2, scale=0.1, gen=g).to(dev), rnd(n // 2, scale=0.1, gen=g).to(dev)
  runs = {}
  for eng in (7, 0):
    prev = lib.cadence_gemm_set_engine(eng)
    try:
      runs[eng] = (ops.linear(a, w), ops.linear(a, w, bias, resid=resid),
                   ops.gated_gelu(a, w, bg, bu))
    finally:
      lib.cadence_gemm_set_engine(prev)
  if m > 4096:
    assert lib.cadence_gemm_engine(m, n, k, 1) == 1, "the plan should take gemm_w4_kernel"
  for what, x, y in zip(("linear", "linear+residual", "gated"), runs[7], runs[0]):
    assert torch.equal(x, y), what
