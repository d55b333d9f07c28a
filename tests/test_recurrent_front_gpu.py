"""The decode recurrent-block front in one launch
(cadence_recurrent_decode_front: y|x projection + Conv1D step + RG-LRU gate
GEMV + scan step, gate = y) against the two launches it replaces
(linear_conv1d_ then rglru_step_; reference modules.py:340-352,
layers.py:478-483, layers.py:345-365 + :175-182).  Bitwise: the y|x output,
the advanced conv state, the fp32 RG-LRU state and the packed y rows, with
rows whose segment position is 0 (state reset), with the RMSNorm pending
(norm on load) and without; twice in a row, so the per-head arrival
counters must come back to zero, and the wait-gave-up flag stays clear."""

import pytest
import torch

from cadence import _lib, layers, ops

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, scale=1.0, gen=None):
  return (torch.randn(*shape, generator=gen) * scale).to(BF)


def _case(dev, m, e, heads, k, gen):
  bw = e // heads
  w = rnd(2 * e, k, scale=k ** -0.5, gen=gen).to(dev)
  bias = rnd(2 * e, scale=0.1, gen=gen).to(dev)
  cw = rnd(4, e, scale=0.5, gen=gen).to(dev)
  cb = rnd(e, scale=0.1, gen=gen).to(dev)
  state = rnd(m, 3, e, gen=gen).to(dev)
  wg = rnd(heads, 2 * bw, bw, scale=bw ** -0.5, gen=gen).to(dev)
  bx = rnd(e, scale=0.1, gen=gen).to(dev)
  ba = rnd(e, scale=0.1, gen=gen).to(dev)
  sp = torch.nn.functional.softplus(rnd(e, gen=gen).float()).to(BF).to(dev)
  pos = torch.randint(0, 5, (m,), generator=gen, dtype=torch.int32)
  pos[0], pos[-1] = 0, 7                      # one reset row, one continuing row
  h = (torch.randn(m, e, generator=gen) * 0.5).to(dev)
  return w, bias, cw, cb, state, (wg, bx, ba, sp), pos.to(dev), h


@pytest.fixture(autouse=True)
def _one_launch(monkeypatch):
  monkeypatch.setattr(ops, "FRONT_ONE_LAUNCH", True)


def _rows(dev, m, k, gen, norm):
  x = rnd(m, k, gen=gen).to(dev)
  if not norm:
    return ops.pack_rows(x)
  n = layers.RMSNorm(k, device=dev, dtype=BF)
  with torch.no_grad():
    n.scale.copy_(rnd(k, scale=0.3, gen=gen).to(dev))
  resid = rnd(m, k, gen=gen).to(dev)
  wr = rnd(k, k, scale=k ** -0.5, gen=gen).to(dev)
  _, lazy = ops.linear_rmsnorm(ops.pack_rows(x), wr, None, resid, n, lazy=True)
  assert lazy.norm is n
  return lazy


@pytest.mark.parametrize("m,e,heads,k,norm", [
    (32, 2560, 10, 2560, True),     # CadenceGemma's recurrent block, bench batch
    (32, 2560, 10, 2560, False),
    (17, 2560, 10, 2560, True),
    (24, 1024, 8, 1280, False),     # bw 128, shorter K
])
def test_recurrent_front_matches_two_launches(dev, m, e, heads, k, norm):
  assert _lib.load().cadence_recurrent_decode_front_plan(m, e, k, heads, e // heads) == 1
  g = torch.Generator().manual_seed(61 + m + e)
  x = _rows(dev, m, k, g, norm)
  w, bias, cw, cb, state, gates, pos, h = _case(dev, m, e, heads, k, g)
  s_ref, s_got, h_ref, h_got = state.clone(), state.clone(), h.clone(), h.clone()
  err = ops.wait_err(dev)
  err.zero_()
  for it in range(2):
    yc = ops.linear_conv1d_(x, w, bias, cw, cb, s_ref)
    y_ref = ops.rglru_step_(yc[:, e:], gates[0], *gates[1:], pos, h_ref, yc[:, :e],
                            packed_out=True)
    y_got = ops.recurrent_decode_front_(x, w, bias, cw, cb, s_got, gates, pos, h_got)
    assert y_got is not None, "shape inside the plan must take the one-launch path"
    torch.cuda.synchronize()
    assert torch.equal(y_got.unpack(), y_ref.unpack()), it
    assert torch.equal(s_got, s_ref), it
    assert torch.equal(h_got, h_ref), it
    cnt = ops._counters(dev, 64 * heads)
    assert int(cnt[:64 * heads].abs().sum()) == 0, it
    assert int(err) == 0
  # the (y, conv1d(x)) output of the same launch
  a, ar, wd, nm = ops._an(x, w)
  s3 = state.clone()
  h3 = h.clone()
  wg = ops.decode_weight(gates[0])
  yx, _ = ops.ops.recurrent_decode_front(a, ar, wd, bias, cw, cb, s3, wg, *gates[1:], pos, h3,
                                         ops._counters(dev, 64 * heads), err, nm is not None,
                                         float(nm.eps) if nm is not None else 0.0)
  want = ops.linear_conv1d_(x, w, bias, cw, cb, state.clone())
  assert torch.equal(yx, want)


def test_recurrent_front_declines_outside_plan(dev):
  """B <= 16 rows (and row-major rows) stay on the two-launch path."""
  g = torch.Generator().manual_seed(5)
  e, heads, k = 2560, 10, 2560
  w, bias, cw, cb, state, gates, pos, h = _case(dev, 8, e, heads, k, g)
  x = ops.pack_rows(rnd(8, k, gen=g).to(dev))
  assert ops.recurrent_decode_front_(x, w, bias, cw, cb, state, gates, pos, h) is None
  assert _lib.load().cadence_recurrent_decode_front_plan(8, e, k, heads, 256) == 0
