"""Prefill RG-LRU with the scan fused in (rglru_scan_fused_kernel) against the
two kernels it replaces (rglru_gates_stream_kernel, then rnn_scan_kernel),
bitwise -- outputs and the fp32 end state -- and, at a smaller batch, against
the CPU oracle's RG-LRU + scan (reference layers.py:145-199, 321-375).

Shapes: the bench's (B = 32 sequences of 319 tokens, 10 blocks of 256), the
C2 batch at a shorter length, ragged sequence lengths (chunks of 16 / 32
steps with a partial last chunk), the 128-wide block instance, with and
without h0 and the y gate (row stride 2E, the [y | x] GEMM output), document
starts inside the sequences (resets)."""

import math

import pytest
import torch

from conftest import assert_close_bf16
from oracle import griffin_ref as R

import cadence
from cadence import ops

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _inputs(b, t, h, bw, seed, with_gate, with_h0, dev):
  g = torch.Generator().manual_seed(seed)
  e = h * bw
  m = b * t
  yx = (torch.randn(m, 2 * e, generator=g)).to(BF).to(dev)
  x = yx[:, e:]                                   # strided, as in the block
  gate = yx[:, :e] if with_gate else None
  w = (torch.randn(h, 2 * bw, bw, generator=g) / math.sqrt(bw)).to(BF).to(dev)
  bx = (torch.randn(e, generator=g) * 0.3).to(BF).to(dev)
  ba = (torch.randn(e, generator=g) * 0.3).to(BF).to(dev)
  sp = torch.rand(e, generator=g).to(BF).to(dev)
  # two documents per sequence: positions restart at a per-row split
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  for i in range(b):
    s = int(torch.randint(1, t, (1,), generator=g))
    pos[i, s:] = torch.arange(t - s, dtype=torch.int32)
  pos = pos.reshape(-1).to(dev)
  h0 = torch.randn(b, e, generator=g).to(dev) if with_h0 else None
  return x, gate, w, bx, ba, sp, pos, h0


@pytest.mark.parametrize("b,t,h,bw,with_gate,with_h0", [
    (32, 319, 10, 256, True, False),      # the bench's recurrent blocks
    (32, 64, 10, 256, True, True),
    (32, 33, 10, 256, False, True),       # 3 chunks of 16, 1-step tail
    (26, 100, 10, 256, True, False),      # 520 workgroups
    (52, 77, 10, 128, True, True),        # the 128-wide instance (32-step chunks)
    (64, 17, 8, 128, False, False)])
def test_rglru_scan_fused_bitwise(dev, b, t, h, bw, with_gate, with_h0):
  x, gate, w, bx, ba, sp, pos, h0 = _inputs(b, t, h, bw, 70 + t, with_gate,
                                            with_h0, dev)
  assert ops.rglru_scan_plan(x, gate, b, t, h, bw)
  y1, hl1 = ops.ops.rglru_scan(x, w, bx, ba, sp, pos, h0, gate, b, t)
  a, nx = ops.ops.rglru_gates(x, w, bx, ba, sp, pos)
  y0, hl0 = ops.ops.rnn_scan(nx, a, None, h0, gate, b, t)
  assert torch.equal(y1, y0)
  assert torch.equal(hl1, hl0)


def test_rglru_scan_fused_vs_oracle(dev):
  """The fused kernel through RecurrentBlock's path against the oracle's
  rg_lru (gate chain op by op) + rnn_scan + `x * y` join, on the CPU."""
  b, t, h, bw = 32, 40, 10, 256
  e = h * bw
  x, gate, w, bx, ba, sp, pos, h0 = _inputs(b, t, h, bw, 91, True, True, dev)
  lru = cadence.RGLRU(e, h, device=dev, dtype=BF)
  g = torch.Generator().manual_seed(92)
  with torch.no_grad():
    lru.input_gate.b.copy_((torch.randn(h, bw, generator=g) * 0.5).to(BF))
    lru.a_gate.b.copy_((torch.randn(h, bw, generator=g) * 0.5).to(BF))
  wp, pbx, pba, psp = lru.packed()
  assert ops.rglru_scan_plan(x, gate, b, t, h, bw)
  y, hl = lru.gates_scan(x, pos, h0, gate, b, t)
  p = {k: v.cpu() for k, v in lru.state_dict().items()}
  xc = x.cpu().reshape(b, t, e)
  y_ref, h_ref = R.rg_lru(xc, pos.cpu().view(b, t), p, "", h0.cpu())
  want = (y_ref * gate.cpu().reshape(b, t, e)).reshape(b * t, e)
  assert_close_bf16(y, want, rtol=2e-2, atol=2e-2, min_equal=0.9, what="fused rg-lru")
  torch.testing.assert_close(hl.cpu(), h_ref, rtol=2e-2, atol=2e-2)


def test_rglru_scan_plan_falls_back_for_small_batches(dev):
  """One sequence (C3) cannot fill the chip with (sequence, block) units:
  the plan declines and gates_scan runs the two kernels (chunked scan)."""
  x, gate, w, bx, ba, sp, pos, h0 = _inputs(1, 319, 10, 256, 93, True, False, dev)
  assert not ops.rglru_scan_plan(x, gate, 1, 319, 10, 256)
  lru = cadence.RGLRU(2560, 10, device=dev, dtype=BF)
  y, hl = lru.gates_scan(x, pos, None, gate, 1, 319)
  assert y.shape == (319, 2560) and hl.shape == (1, 2560)
