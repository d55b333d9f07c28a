"""Decode activation layout ("packed rows", include/cadence_kernels.h).

Every decode-side producer's packed output must equal pack_rows() of its
row-major output, and every consumer must give bit-identical results on
packed vs row-major activations (same engine, same summation order).
"""

import math

import pytest
import torch

import cadence
from cadence import ops

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, scale=1.0, gen=None):
  return (torch.randn(*shape, generator=gen) * scale).to(BF)


@pytest.mark.parametrize("m", [32, 17, 5])
def test_packed_rows_producers_and_consumers(dev, m):
  g = torch.Generator().manual_seed(21)
  k, n, f = 2560, 512, 256
  x = rnd(m, k, gen=g).to(dev)
  xp = ops.pack_rows(x)
  assert torch.equal(xp.unpack(), x)
  # producer: RMSNorm
  scale = rnd(k, scale=0.2, gen=g).to(dev)
  rn = ops.rmsnorm(x, scale, 1e-6, packed=True)
  assert isinstance(rn, ops.PackedRows)
  assert torch.equal(rn.unpack(), ops.rmsnorm(x, scale, 1e-6))
  # consumer: linear (+ bias + residual)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g).to(dev)
  bias = rnd(n, scale=0.1, gen=g).to(dev)
  resid = rnd(m, n, gen=g).to(dev)
  assert torch.equal(ops.linear(xp, w, bias, resid=resid),
                     ops.linear(x, w, bias, resid=resid))
  # consumer + producer: split-K residual GEMM fused with the next RMSNorm
  wk = rnd(n, 7680, scale=1 / 90, gen=g).to(dev)
  xk = rnd(m, 7680, gen=g).to(dev)
  norm = cadence.layers.RMSNorm(n, device=dev, dtype=BF)
  o1, n1 = ops.linear_rmsnorm(ops.pack_rows(xk), wk, bias, resid, norm)
  o2, n2 = ops.linear_rmsnorm(xk, wk, bias, resid, norm, packed_out=False)
  assert isinstance(n1, ops.PackedRows)
  assert torch.equal(o1, o2) and torch.equal(n1.unpack(), n2)
  # consumer + producer: gated GELU
  wg = rnd(2 * f, k, scale=1 / math.sqrt(k), gen=g).to(dev)
  bg, bu = rnd(f, scale=0.1, gen=g).to(dev), rnd(f, scale=0.1, gen=g).to(dev)
  g1 = ops.gated_gelu(xp, wg, bg, bu)
  g2 = ops.gated_gelu(x, wg, bg, bu, packed_out=False)
  assert isinstance(g1, ops.PackedRows) and torch.equal(g1.unpack(), g2)
  # consumers: logits (+ soft-cap, argmax)
  emb = rnd(1024, k, scale=0.05, gen=g).to(dev)
  l1, a1 = ops.logits_argmax(xp, emb, 30.0, True)
  l2, a2 = ops.logits_argmax(x, emb, 30.0, True)
  assert torch.equal(l1, l2) and torch.equal(a1, a2)
  assert torch.equal(ops.gemm_logits(xp, emb, 30.0), ops.gemm_logits(x, emb, 30.0))
  # producer: RG-LRU decode step
  h_, bw = 10, 256
  e = h_ * bw
  yx = rnd(m, 2 * e, gen=g).to(dev)
  wr = rnd(h_, 2 * bw, bw, scale=1 / 16, gen=g).to(dev)
  bx, ba = rnd(e, scale=0.3, gen=g).to(dev), rnd(e, scale=0.3, gen=g).to(dev)
  sp = torch.rand(e, generator=g).to(BF).to(dev)
  pos = torch.randint(0, 3, (m,), generator=g, dtype=torch.int32).to(dev)
  h0 = torch.randn(m, e, generator=g).to(dev)
  ha, hb = h0.clone(), h0.clone()
  y1 = ops.rglru_step_(x, wr, bx, ba, sp, pos, ha, yx[:, :e])
  y2 = ops.rglru_step_(x, wr, bx, ba, sp, pos, hb, yx[:, :e], packed_out=False)
  assert isinstance(y1, ops.PackedRows)
  assert torch.equal(y1.unpack(), y2) and torch.equal(ha, hb)


def test_packed_rows_decode_attention(dev):
  g = torch.Generator().manual_seed(22)
  b, h, hd, window = 3, 10, 256, 64
  ck = rnd(b, window, 1, hd, gen=g).to(dev)
  cv = rnd(b, window, 1, hd, gen=g).to(dev)
  nt = torch.tensor([5, 63, 100], dtype=torch.int32, device=dev)
  q = rnd(b, h * hd, gen=g).to(dev)
  kn, vn = rnd(b, hd, gen=g).to(dev), rnd(b, hd, gen=g).to(dev)
  ck2, cv2, nt2 = ck.clone(), cv.clone(), nt.clone()
  want = ops.ops.local_attention_decode_(q, kn, vn, ck, cv, nt, h)
  got = ops.local_attention_decode_(q, kn, vn, ck2, cv2, nt2, h)
  assert isinstance(got, ops.PackedRows)
  assert torch.equal(got.unpack(), want)
  assert torch.equal(ck, ck2) and torch.equal(cv, cv2) and torch.equal(nt, nt2)
