"""The reference's own layer / module test grids on the GPU path.

recurrentgemma/torch/layers_test.py:96-172 (RGLRU, Conv1D) and
modules_test.py:77-116 (LocalAttentionBlock) compare torch against jax with
test_utils.numerically_compare_modules (test_utils.py:59-107): a forward over
[1, seq, width] with two-document positions (two halves, each from 0), then
two single-token steps from the returned cache.  Here the HIP path is held
to the CPU oracle the same way, at bf16 with the reference's bf16 tolerance
(rtol 1e-2, atol 3e-2, layers_test.py:131,170), on every grid point --
including the shapes the tuned kernels do not cover (RG-LRU heads 8 wide,
attention head dims 16 and 1024, Conv1D temporal width 8), and the cached
multi-token step of modules.py:206-225 (n_fill == window).
"""

import pytest
import torch

from conftest import assert_close_bf16
from oracle import griffin_ref as R

import cadence

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
TOL = dict(rtol=1e-2, atol=3e-2)


def two_doc_pos(t):
  half = torch.arange(t // 2, dtype=torch.int32)
  return torch.cat([half, half])[None]


def _params(mod, gen, scale=0.5):
  """Random (non-identity) parameters for `mod`, copied into it; returns the
  CPU dict the oracle reads."""
  p = {}
  with torch.no_grad():
    for name, t in mod.named_parameters():
      v = (torch.randn(t.shape, generator=gen) * scale /
           max(1.0, t.shape[-1] ** 0.5)).to(t.dtype)
      if name.endswith("a_param"):
        v = (torch.rand(t.shape, generator=gen) * 2 - 3).to(t.dtype)
      t.copy_(v.to(t.device))
      p[name] = v
  return p


def _cache_close(cache, ref):
  """Ring buffers: fill counters exact; keys / values are projections (a
  GEMM's accumulation order differs from the oracle's F.linear) and keys
  also carry RoPE's sin / cos rounding: the bf16 tolerance, and the slots
  that hold nothing (zero in the oracle) must be zero here too."""
  assert torch.equal(cache.num_tokens.cpu(), ref["num_tokens"])
  for got, want, what in ((cache.keys, ref["keys"], "keys"),
                          (cache.values, ref["values"], "values")):
    got = got.cpu().view(want.shape)
    assert_close_bf16(got, want, **TOL, what=f"cache {what}")
    empty = (want == 0).all(dim=-1)
    assert bool((got[empty] == 0).all()), f"cache {what}: empty slots"


@pytest.mark.parametrize("width", [128, 1024])
@pytest.mark.parametrize("num_heads", [1, 8])
@pytest.mark.parametrize("window", [8, 16])
def test_local_attention_grid(dev, width, num_heads, window):
  """modules_test.py:77-116: seq 64, forward then 2 cached steps."""
  g = torch.Generator().manual_seed(12413166 + width + num_heads + window)
  blk = cadence.LocalAttentionBlock(width, num_heads, window, device=dev, dtype=BF)
  p = _params(blk, g)
  t = 64
  x = (torch.randn(1, t, width, generator=g)).to(BF)
  pos = two_doc_pos(t)
  want, cache_ref = R.local_attention(x, pos, p, "", num_heads, window)
  got, cache = blk(x.to(dev), pos.to(dev))
  assert_close_bf16(got, want, **TOL, what="attention forward")
  _cache_close(cache, cache_ref)
  y = torch.randn(1, 2, width, generator=g).to(BF)
  for i in range(2):
    sp = pos[:, -1:] + 1 + i
    want, cache_ref = R.local_attention(y[:, i:i + 1], sp, p, "", num_heads,
                                        window, cache_ref)
    got, cache = blk(y[:, i:i + 1].to(dev), sp.to(dev), cache)
    assert_close_bf16(got, want, **TOL, what=f"attention step {i}")
    _cache_close(cache, cache_ref)


@pytest.mark.parametrize("hd,num_heads,chunk", [(256, 2, 16), (16, 8, 24)])
def test_attention_cached_prompt_chunk(dev, hd, num_heads, chunk):
  """modules.py:206-225, n_fill == window: a multi-token step (t >= window)
  against an existing cache attends over [ring | new rows] with the cache
  mask and returns a fresh cache from the new rows."""
  window = 16
  width = hd * num_heads
  g = torch.Generator().manual_seed(77 + hd)
  blk = cadence.LocalAttentionBlock(width, num_heads, window, device=dev, dtype=BF)
  p = _params(blk, g)
  b, t0 = 2, 20
  x = torch.randn(b, t0, width, generator=g).to(BF)
  pos = torch.arange(t0, dtype=torch.int32)[None].repeat(b, 1)
  _, cache_ref = R.local_attention(x, pos, p, "", num_heads, window)
  _, cache = blk(x.to(dev), pos.to(dev))
  y = torch.randn(b, chunk, width, generator=g).to(BF)
  sp = torch.arange(t0, t0 + chunk, dtype=torch.int32)[None].repeat(b, 1)
  want, new_ref = R.local_attention(y, sp, p, "", num_heads, window, cache_ref)
  got, new = blk(y.to(dev), sp.to(dev), cache)
  assert_close_bf16(got, want, **TOL, what="cached chunk")
  _cache_close(new, new_ref)
  with pytest.raises(NotImplementedError):   # 1 < t < window (modules.py:224)
    blk(y[:, :3].to(dev), sp[:, :3].to(dev), cache)
  # without a returned cache the reference never reaches that raise: it
  # attends over [ring | 3 new rows] with the cache mask (modules.py:439-451)
  want, none_ref = R.local_attention(y[:, :3], sp[:, :3], p, "", num_heads,
                                     window, cache_ref, return_cache=False)
  got, none = blk(y[:, :3].to(dev), sp[:, :3].to(dev), cache, return_cache=False)
  assert none is None and none_ref is None
  assert_close_bf16(got, want, **TOL, what="cached 3-token step, no cache")


@pytest.mark.parametrize("width", [128, 1024])
@pytest.mark.parametrize("num_heads", [1, 16])
@pytest.mark.parametrize("seq_len", [32, 128])
def test_rglru_grid(dev, width, num_heads, seq_len):
  """layers_test.py:96-133: forward then 2 cached steps (width 128 x 16
  heads is 8 wide: merged block-diagonally for the gate GEMM)."""
  g = torch.Generator().manual_seed(9018323 + width + num_heads + seq_len)
  lru = cadence.RGLRU(width, num_heads, device=dev, dtype=BF)
  p = _params(lru, g)
  x = torch.randn(1, seq_len, width, generator=g).to(BF)
  pos = two_doc_pos(seq_len)
  want, h_ref = R.rg_lru(x, pos, p, "")
  got, h = lru(x.to(dev), pos.to(dev))
  assert_close_bf16(got, want, **TOL, what="rglru forward")
  torch.testing.assert_close(h.cpu(), h_ref, **TOL)
  y = torch.randn(1, 2, width, generator=g).to(BF)
  for i in range(2):
    sp = pos[:, -1:] + 1 + i
    want, h_ref = R.rg_lru(y[:, i:i + 1], sp, p, "", h_ref)
    got, h = lru(y[:, i:i + 1].to(dev), sp.to(dev), h)
    assert_close_bf16(got, want, **TOL, what=f"rglru step {i}")
    torch.testing.assert_close(h.cpu(), h_ref, **TOL)


@pytest.mark.parametrize("width", [128, 1024])
@pytest.mark.parametrize("temporal_width", [4, 8])
def test_conv1d_grid(dev, width, temporal_width):
  """layers_test.py:136-172 (seq 32): bit-exact with the oracle, prefill
  and 2 cached steps, both temporal widths."""
  g = torch.Generator().manual_seed(9018323 + width + temporal_width)
  conv = cadence.Conv1D(width, temporal_width, device=dev, dtype=BF)
  p = _params(conv, g, scale=1.0)
  x = torch.randn(1, 32, width, generator=g).to(BF)
  pos = two_doc_pos(32)
  want, c_ref = R.conv1d(x, pos, p["w"], p["b"])
  got, c = conv(x.to(dev), pos.to(dev))
  assert torch.equal(got.cpu(), want) and torch.equal(c.cpu(), c_ref)
  y = torch.randn(1, 2, width, generator=g).to(BF)
  for i in range(2):
    sp = pos[:, -1:] + 1 + i
    want, c_ref = R.conv1d(y[:, i:i + 1], sp, p["w"], p["b"], c_ref)
    got, c = conv(y[:, i:i + 1].to(dev), sp.to(dev), c)
    assert torch.equal(got.cpu(), want) and torch.equal(c.cpu(), c_ref)


@pytest.mark.parametrize("temporal_width", [4, 8])
@pytest.mark.parametrize("start", [3, 5, 6, 7])
def test_conv1d_cache_late_document(dev, temporal_width, start):
  """Appendix A Q4: a document starting `start` tokens before the end.  The
  reference zeroes masked rows of x in place (layers.py:506,524) before it
  caches x[:, 1-width:] (:542), so a width-8 cache loses rows L-7..L-4 ahead
  of the new document; width 4 never does.  Bit-exact with the oracle."""
  g = torch.Generator().manual_seed(55 + temporal_width + start)
  width, L = 128, 32
  conv = cadence.Conv1D(width, temporal_width, device=dev, dtype=BF)
  p = _params(conv, g, scale=1.0)
  x = torch.randn(2, L, width, generator=g).to(BF)
  pos = torch.arange(L, dtype=torch.int32)[None].repeat(2, 1)
  pos[0, L - start:] = torch.arange(start, dtype=torch.int32)   # new document
  want, c_ref = R.conv1d(x, pos, p["w"], p["b"])
  got, c = conv(x.to(dev), pos.to(dev))
  assert torch.equal(got.cpu(), want) and torch.equal(c.cpu(), c_ref)
  if temporal_width == 8 and start <= 5:
    assert not torch.equal(c_ref[0], x[0, 1 - temporal_width:])   # Q4 reached

