"""Split-K form of the prefill GEMM engine (small M: one image / one prompt,
cadence_gemm_big_splits > 1): EpiPartial fp32 split partials, then the real
epilogue on the split-order sums.  Checked against fp32 references at the
reference's bf16 tolerance (layers_test.py:131,170), bit-reproducible, and
the split plan itself at the C3 shapes."""

import math

import pytest
import torch
import torch.nn.functional as F

from cadence import _lib, ops
from conftest import assert_close_bf16

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, scale=1.0, gen=None):
  return (torch.randn(*shape, generator=gen) * scale).to(BF)


def test_split_plan_at_c3_shapes():
  lib = _lib.load()
  # one 224-px image through the towers: 261 / 256 tokens
  assert lib.cadence_gemm_big_splits(261, 3072, 1024, 1) > 1
  assert lib.cadence_gemm_big_splits(256, 1152, 4352, 1) > 1
  # one 319-token prompt through Griffin
  assert lib.cadence_gemm_big_splits(319, 2560, 7680, 1) > 1
  assert lib.cadence_gemm_big_splits(319, 15360, 2560, 1) > 1
  # the bench shapes (32 images) keep one pass
  assert lib.cadence_gemm_big_splits(32 * 261, 1024, 1024, 1) == 1
  assert lib.cadence_gemm_big_splits(32 * 319, 15360, 2560, 1) == 1


@pytest.mark.parametrize("m,n,k,act", [(261, 3072, 1024, 0), (261, 4096, 1024, 1),
                                       (319, 2560, 7680, 0), (256, 1152, 4352, 0)])
def test_split_linear(dev, m, n, k, act):
  assert _lib.load().cadence_gemm_big_splits(m, n, k, 1) > 1
  g = torch.Generator().manual_seed(21)
  a = rnd(m, k, gen=g)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g)
  bias = rnd(n, scale=0.1, gen=g)
  resid = rnd(m, n, gen=g)
  want = F.linear(a.float(), w.float(), bias.float())
  if act == 1:
    want = F.gelu(want.to(BF).float())
  got = [ops.linear(a.to(dev), w.to(dev), bias.to(dev), act=act) for _ in range(3)]
  assert_close_bf16(got[0], want.to(BF), rtol=1e-2, atol=1e-2, what="split linear")
  assert torch.equal(got[0], got[1]) and torch.equal(got[0], got[2])
  got_r = ops.linear(a.to(dev), w.to(dev), bias.to(dev), resid=resid.to(dev))
  want_r = (F.linear(a.float(), w.float(), bias.float()).to(BF) + resid)
  assert_close_bf16(got_r, want_r, rtol=1e-2, atol=2e-2, what="split residual")


def test_split_gated_gelu(dev):
  m, f, k = 319, 7680, 2560
  g = torch.Generator().manual_seed(22)
  a = rnd(m, k, gen=g)
  wp = rnd(2 * f, k, scale=1 / math.sqrt(k), gen=g)
  bg, bu = rnd(f, scale=0.1, gen=g), rnd(f, scale=0.1, gen=g)
  wv = wp.float().view(f // 32, 2, 32, k)
  gate = (a.float() @ wv[:, 0].reshape(f, k).T).to(BF).float() + bg.float()
  up = (a.float() @ wv[:, 1].reshape(f, k).T).to(BF).float() + bu.float()
  want = (F.gelu(gate.to(BF).float(), approximate="tanh").to(BF).float() *
          up.to(BF).float()).to(BF)
  got = ops.ops.gated_gelu(a.to(dev), wp.to(dev), bg.to(dev), bu.to(dev))
  assert_close_bf16(got, want, rtol=2e-2, atol=2e-2, what="split gated gelu")


def test_split_vit_residual(dev):
  m, n, k = 261, 1024, 4096
  g = torch.Generator().manual_seed(23)
  a = rnd(m, k, gen=g)
  w = rnd(n, k, scale=1 / math.sqrt(k), gen=g)
  bias = rnd(n, scale=0.1, gen=g)
  gamma = rnd(n, scale=0.5, gen=g)
  resid = torch.randn(m, n, generator=g)
  want = resid + gamma.float() * F.linear(a.float(), w.float(), bias.float())
  r = resid.to(dev)
  ops.ops.vit_residual_(a.to(dev), w.to(dev), bias.to(dev), gamma.to(dev), r)
  torch.testing.assert_close(r.cpu(), want, rtol=2e-2, atol=2e-2)
