"""The captured decode step's one-launch tail (cadence_logits_argmax_tail)
against the three launches it replaces in the eager step: logits_argmax's
greedy argmax, decode_advance_ (examples/cadence_sampler.py:131-151 and the
done test of recurrentgemma/torch/sampler.py:217-223) and the next token's
embedding in both layouts (embed_packed_; modules.py:994-1001).  Bitwise,
including the EOS flags (a row already done, a row that emits EOS now), the
step counter and the arrival counter left at zero for the next launch."""

import pytest
import torch

from cadence import ops

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _state(b, steps, dev):
  return dict(buf=torch.full((b, steps), 7, dtype=torch.int32, device=dev),
              step=torch.full((1,), 3, dtype=torch.int32, device=dev),
              pos=torch.arange(b, dtype=torch.int32, device=dev) + 40,
              cur=torch.zeros(b, dtype=torch.int32, device=dev),
              done=torch.zeros(b + 1, dtype=torch.int32, device=dev))


@pytest.mark.parametrize("b", [1, 5, 32])
def test_logits_argmax_tail_matches_three_launches(dev, b):
  g = torch.Generator().manual_seed(31 + b)
  d, v, steps, cap = 256, 4096, 8, 30.0
  x = (torch.randn(b, d, generator=g) * 0.5).to(BF).to(dev)
  emb = (torch.randn(v, d, generator=g) * 0.05).to(BF).to(dev)
  scale = float(torch.tensor(d ** 0.5).to(BF))
  _, want_next = ops.logits_argmax(x, emb, cap, False)
  pad = 0
  eos = int(want_next[0])                    # row 0 emits EOS at this step
  ref, got = _state(b, steps, dev), _state(b, steps, dev)
  if b > 2:
    ref["done"][2] = 1                       # row 2 finished earlier: pad
    got["done"][2] = 1
  eos_args = (eos, pad, 1)
  # eager: three launches
  ops.ops.decode_advance_(want_next, ref["buf"], ref["step"], ref["pos"], ref["cur"],
                          ref["done"], *eos_args)
  x_ref = torch.empty(b, d, dtype=BF, device=dev)
  xp_ref = ops.packed_empty(b, d, dev)
  ops.ops.embed_packed_(ref["cur"], emb, scale, x_ref, xp_ref)
  # one tail launch, twice in a row: the arrival counter must come back to 0
  counter = torch.zeros(1, dtype=torch.int32, device=dev)
  x_got = torch.zeros(b, d, dtype=BF, device=dev)
  xp_got = ops.packed_empty(b, d, dev).zero_()
  tail = dict(got, eos_args=eos_args, counter=counter, x=x_got, xp=xp_got, scale=scale)
  nxt = ops.logits_argmax_tail(x, emb, cap, tail)
  torch.cuda.synchronize()
  assert torch.equal(nxt, want_next)
  for k in ("buf", "step", "pos", "cur", "done"):
    assert torch.equal(got[k], ref[k]), k
  assert torch.equal(x_got, x_ref)
  # the packed rows (the layout's padding rows past b are not written)
  assert torch.equal(ops.PackedRows(xp_got, b, d).unpack(), ops.PackedRows(xp_ref, b, d).unpack())
  assert int(counter) == 0
  assert int(got["done"][0]) == 1 and int(got["step"]) == 4
  # the second launch continues from the advanced state
  ops.ops.decode_advance_(want_next, ref["buf"], ref["step"], ref["pos"], ref["cur"],
                          ref["done"], *eos_args)
  ops.logits_argmax_tail(x, emb, cap, tail)
  torch.cuda.synchronize()
  for k in ("buf", "step", "pos", "cur", "done"):
    assert torch.equal(got[k], ref[k]), k
  assert int(counter) == 0
