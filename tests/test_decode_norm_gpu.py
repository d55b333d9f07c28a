"""Decode residual projections with the RMSNorm deferred to the consuming
GEMV (cadence_gemm_linear_residual_rows + norm-on-load in
cadence_gemm_linear_conv1d / cadence_qkv_rope_decode /
cadence_gemm_gated_gelu).

* The residual output and its unnormalised packed copy are bit-identical to
  the two-kernel split-K path (same split-order sums, same roundings).
* A consumer fed the pending-norm rows (norm scale folded into its weight,
  the rows' rsqrt applied to the fp32 dot products: cadence_kernels.h
  "Deferred RMSNorm") matches the same consumer fed rows normalised by the
  standalone RMSNorm kernel at the reference's bf16 tolerance
  (layers_test.py:131,170), and is at least as close to an fp32 evaluation
  of the op as that reference-rounding path (it skips two per-element bf16
  roundings).
"""

import pytest
import torch

from cadence import layers, ops

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, scale=1.0, gen=None):
  return (torch.randn(*shape, generator=gen) * scale).to(BF)


def _norm(dev, width, gen):
  n = layers.RMSNorm(width, device=dev, dtype=BF)
  with torch.no_grad():
    n.scale.copy_(rnd(width, scale=0.3, gen=gen).to(dev))
  return n


def _close(got, want, frac=0.25, tol=2e-2):
  """Allclose at the reference bf16 tolerance and mostly bit-equal."""
  got, want = got.float(), want.float()
  torch.testing.assert_close(got, want, rtol=tol, atol=tol)
  eq = (got == want).float().mean().item()
  assert eq >= frac, f"only {eq:.4f} bit-equal"


@pytest.mark.parametrize("m,k", [(32, 2560), (32, 7680), (20, 2560), (1, 7680), (5, 2560),
                                 (1, 2560)])
def test_residual_rows_match_two_kernel_path(dev, m, k):
  g = torch.Generator().manual_seed(41)
  n = 2560
  x = rnd(m, k, gen=g).to(dev)
  w = rnd(n, k, scale=k ** -0.5, gen=g).to(dev)
  bias = rnd(n, scale=0.1, gen=g).to(dev)
  resid = rnd(m, n, gen=g).to(dev)
  norm = _norm(dev, n, g)
  a = ops.pack_rows(x)
  out1, n1 = ops.linear_rmsnorm(a, w, bias, resid, norm)
  out2, r2 = ops.linear_rmsnorm(a, w, bias, resid, norm, lazy=True)
  assert isinstance(r2, ops.PackedRows) and r2.norm is norm
  if k == 2560:
    # the output projection's unsplit kernel (gemm_resid_pipe_kernel, one or
    # two 16-row tiles): one fp32 chain over all of K instead of the
    # split-order sums
    _close(out2, out1, frac=0.99)
  else:
    assert torch.equal(out1, out2)
  assert torch.equal(r2.unpack(), out2)
  _close(r2.normalised().unpack(), n1.unpack(), frac=0.999)
  # repeated launches reuse the (self-resetting) arrival counters
  for _ in range(3):
    out3, r3 = ops.linear_rmsnorm(a, w, bias, resid, norm, lazy=True)
    assert torch.equal(out3, out2) and torch.equal(r3.unpack(), r2.unpack())


def _rows(dev, m, gen):
  """(pending-norm rows, the same rows normalised by the RMSNorm kernel,
  the fp32 RMSNorm of the rows)."""
  n, k = 2560, 2560
  x = rnd(m, k, gen=gen).to(dev)
  w = rnd(n, k, scale=k ** -0.5, gen=gen).to(dev)
  resid = rnd(m, n, gen=gen).to(dev)
  norm = _norm(dev, n, gen)
  _, lazy = ops.linear_rmsnorm(ops.pack_rows(x), w, None, resid, norm, lazy=True)
  assert lazy.norm is norm
  r = lazy.src.float()
  f32 = r * torch.rsqrt((r * r).mean(-1, keepdim=True) + norm.eps) * (
      norm.scale.float() + 1.0)
  return lazy, lazy.normalised(), f32


def _no_worse(got, want, ref, slack=1.25):
  """got is no further from the fp32 evaluation `ref` than want is."""
  e_got = ((got.float() - ref).norm() / ref.norm()).item()
  e_want = ((want.float() - ref).norm() / ref.norm()).item()
  assert e_got <= slack * e_want + 1e-4, (e_got, e_want)


@pytest.mark.parametrize("m", [32, 13])
def test_gated_gelu_norm_on_load(dev, m):
  g = torch.Generator().manual_seed(43)
  lazy, normed, f32 = _rows(dev, m, g)
  f, k = 7680, 2560
  wp = rnd(2 * f, k, scale=k ** -0.5, gen=g).to(dev)
  bg = rnd(f, scale=0.1, gen=g).to(dev)
  bu = rnd(f, scale=0.1, gen=g).to(dev)
  got = ops.gated_gelu(lazy, wp, bg, bu).unpack()
  want = ops.gated_gelu(normed, wp, bg, bu).unpack()
  _close(got, want, frac=0.25, tol=3e-2)   # gelu(g) * u: two roundings compound
  # fp32 evaluation; packed rows: 32 gate rows then 32 up rows per 64
  wv = wp.float().view(f // 32, 2, 32, k)
  gate = f32 @ wv[:, 0].reshape(f, k).T + bg.float()
  up = f32 @ wv[:, 1].reshape(f, k).T + bu.float()
  ref = torch.nn.functional.gelu(gate, approximate="tanh") * up
  _no_worse(got, want, ref)


@pytest.mark.parametrize("m", [32, 7])
def test_linear_conv1d_norm_on_load(dev, m):
  g = torch.Generator().manual_seed(47)
  lazy, normed, f32 = _rows(dev, m, g)
  k, e, tw = 2560, 2560, 4
  w = rnd(2 * e, k, scale=k ** -0.5, gen=g).to(dev)
  bias = rnd(2 * e, scale=0.1, gen=g).to(dev)
  cw = rnd(tw, e, scale=0.5, gen=g).to(dev)
  cb = rnd(e, scale=0.1, gen=g).to(dev)
  state = rnd(m, tw - 1, e, gen=g).to(dev)
  s1, s2 = state.clone(), state.clone()
  got = ops.linear_conv1d_(lazy, w, bias, cw, cb, s1)
  want = ops.linear_conv1d_(normed, w, bias, cw, cb, s2)
  _close(got, want)
  _close(s1, s2)
  _no_worse(got[:, :e], want[:, :e], f32 @ w[:e].float().T + bias[:e].float())


@pytest.mark.parametrize("m", [32, 5])
def test_qkv_rope_decode_norm_on_load(dev, m):
  g = torch.Generator().manual_seed(53)
  lazy, normed, _ = _rows(dev, m, g)
  h, hd, k = 10, 256, 2560
  w = rnd((h + 2) * hd, k, scale=k ** -0.5, gen=g).to(dev)
  pos = torch.randint(0, 3000, (m,), generator=g, dtype=torch.int32).to(dev)
  wp = w[ops.qkv_rope_permutation(h, hd, dev)].contiguous()
  got = ops.qkv_rope_decode(lazy, wp, pos, h, hd)
  want = ops.qkv_rope_decode(normed, wp, pos, h, hd)
  for a, b in zip(got, want):
    _close(a, b)


def test_pending_norm_rows_materialise_for_other_consumers(dev):
  """A consumer that cannot normalise on load (plain linear) gets the rows
  through the standalone norm: identical to passing normalised rows."""
  g = torch.Generator().manual_seed(59)
  lazy, normed, _ = _rows(dev, 32, g)
  w = rnd(512, 2560, scale=2560 ** -0.5, gen=g).to(dev)
  assert torch.equal(ops.linear(lazy, w), ops.linear(normed, w))


@pytest.mark.parametrize("m", [32, 20, 16, 7, 1])
def test_gated_pipe_kernel_matches_stream_kernel(dev, m):
  """The two-pair pipelined decode up-projection (packed rows: one 16-row
  tile up to 16 rows -- the B = 1 decode of C3 -- two up to 32) sums in the
  one-pair stream kernel's order: bit-identical outputs at the 2B model's
  shape (F = 7680, K = 2560)."""
  g = torch.Generator().manual_seed(61)
  f, k = 7680, 2560
  x = rnd(m, k, gen=g).to(dev)
  wp = rnd(2 * f, k, scale=k ** -0.5, gen=g).to(dev)
  bg = rnd(f, scale=0.1, gen=g).to(dev)
  bu = rnd(f, scale=0.1, gen=g).to(dev)
  got = ops.gated_gelu(ops.pack_rows(x), wp, bg, bu)          # pipelined kernel
  want = ops.gated_gelu(x, wp, bg, bu, packed_out=False)       # row-major A: stream kernel
  assert torch.equal(got.unpack(), want)
