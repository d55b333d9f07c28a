"""Decode-step fusions: each fused launch must be bit-identical to the
unfused op sequence it replaces (same kernels' arithmetic, same roundings).
"""

import pytest
import torch

from cadence import ops

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, scale=1.0, gen=None):
  return (torch.randn(*shape, generator=gen) * scale).to(BF)


@pytest.mark.parametrize("m,packed", [(32, True), (17, True), (5, False)])
def test_linear_conv1d_matches_linear_then_conv_step(dev, m, packed):
  """cadence_gemm_linear_conv1d == cadence_gemm_linear + cadence_conv1d
  (decode, L == 1), including the in-place conv state shift."""
  g = torch.Generator().manual_seed(31)
  k, e, tw = 2560, 2560, 4
  x = rnd(m, k, gen=g).to(dev)
  w = rnd(2 * e, k, scale=k ** -0.5, gen=g).to(dev)
  bias = rnd(2 * e, scale=0.1, gen=g).to(dev)
  cw = rnd(tw, e, scale=0.5, gen=g).to(dev)
  cb = rnd(e, scale=0.1, gen=g).to(dev)
  state = rnd(m, tw - 1, e, gen=g).to(dev)
  s_ref, s_got = state.clone(), state.clone()
  a = ops.pack_rows(x) if packed else x
  yx = ops.linear(a, w, bias)
  conv = ops.ops.conv1d_step_(yx[:, e:], cw, cb, s_ref)
  got = ops.linear_conv1d_(a, w, bias, cw, cb, s_got)
  assert torch.equal(got[:, :e], yx[:, :e])
  assert torch.equal(got[:, e:], conv)
  assert torch.equal(s_got, s_ref)


def test_linear_conv1d_rejects_prefill_rows(dev):
  k, e = 256, 128
  x = torch.zeros(40, k, dtype=BF, device=dev)
  w = torch.zeros(2 * e, k, dtype=BF, device=dev)
  cw = torch.zeros(4, e, dtype=BF, device=dev)
  cb = torch.zeros(e, dtype=BF, device=dev)
  st = torch.zeros(40, 3, e, dtype=BF, device=dev)
  with pytest.raises(RuntimeError):
    ops.ops.gemm_linear_conv1d_(x, w, None, cw, cb, st)


@pytest.mark.parametrize("m,packed", [(32, True), (9, False)])
def test_qkv_rope_decode_matches_linear_then_rope(dev, m, packed):
  """cadence_qkv_rope_decode (permuted weight, RoPE in the epilogue) ==
  cadence_gemm_linear + cadence_rope_qkv, bit for bit, incl. positions
  outside the sin/cos table (computed on the fly) and negative positions."""
  g = torch.Generator().manual_seed(33)
  h, hd, k = 10, 256, 2560
  x = rnd(m, k, gen=g).to(dev)
  w = rnd((h + 2) * hd, k, scale=k ** -0.5, gen=g).to(dev)
  pos = torch.randint(0, 3000, (m,), generator=g, dtype=torch.int32)
  pos[0] = 5000                      # past the table
  pos[-1] = -1                       # padding position
  pos = pos.to(dev)
  table = ops.rope_table(dev, hd)
  a = ops.pack_rows(x) if packed else x
  qkv = ops.linear(a, w)
  q1, k1, v1 = ops.ops.rope_qkv(qkv, pos, h, hd, table)
  wp = w[ops.qkv_rope_permutation(h, hd, dev)].contiguous()
  q2, k2, v2 = ops.qkv_rope_decode(a, wp, pos, h, hd)
  assert torch.equal(q1, q2) and torch.equal(k1, k2) and torch.equal(v1, v2)
