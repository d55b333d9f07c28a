"""Sampler stopping and sampling modes on the GPU.

Default EOS handling is the reference's loop (recurrentgemma/torch/
sampler.py:177-187, 209-225, 291-300): `done_now = torch.equal(next_token,
eos)` with eos a [1] tensor, so a batch of one row stops after a DECODE step
samples EOS (the token sampled from the prompt, column 0, is never tested;
the rest of the buffer stays pad) and rows of a larger batch never stop.
`_reference_loop` below restates that loop on a free run's tokens.

`Sampler(eos_per_row=True)` is the opt-in per-row mode, flags kept on the
device by `decode_advance`: once a row emits EOS (column 0 included) the
rest of its buffer is pad, and the host stops issuing steps once every row
is done (it reads the flag a few steps late; late steps only write pad).
Categorical sampling (`greedy_sampling=False`, sampler.py:130-136).
"""

import pytest
import torch

import cadence
from test_model_gpu import MockVocab, make_model, small_config

pytestmark = pytest.mark.gpu


class EosVocab(MockVocab):
  def __init__(self, eos):
    self._eos = eos

  def eos_id(self):
    return self._eos


def _reference_loop(free, eos, pad):
  """recurrentgemma/torch/sampler.py:209-225 on the free run's tokens: the
  while loop runs while step < total - 1 and not all(done); done |=
  torch.equal(next_token [B], eos [1]), which only a 1-row batch can meet."""
  b, steps = free.shape
  want = torch.full_like(free, pad)
  want[:, 0] = free[:, 0]                       # sampled from the prompt
  done = False
  step = 0
  while step < steps - 1 and not done:
    nxt = free[:, step + 1]
    want[:, step + 1] = nxt
    done = done or torch.equal(nxt, torch.tensor([eos], dtype=nxt.dtype))
    step += 1
  return want


def _expected_with_eos(free, eos, pad):
  want = free.clone()
  for r in range(want.shape[0]):
    hit = (want[r] == eos).nonzero()
    if len(hit):
      want[r, int(hit[0]) + 1:] = pad
  return want


@pytest.mark.parametrize("use_graph", [True, False])
def test_eos_stop_pads_rows_and_graph_reuse(dev, use_graph):
  cfg = small_config(vocab=64, window=32)
  m, _ = make_model(dev, cfg, seed=31)
  b, steps = 4, 40
  runs = []
  for seed, t in ((1, 20), (2, 11)):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(3, cfg.vocab_size, (b, t), generator=g, dtype=torch.int32)
    runs.append((tok, torch.full((b,), t, dtype=torch.int32)))
  free = [cadence.Sampler(m, MockVocab(), use_graph=False).generate(
      tok, lens, steps).tokens_buffer.cpu() for tok, lens in runs]
  # the most frequent generated token of the first run acts as EOS
  eos = int(torch.mode(free[0].flatten()).values)
  s = cadence.Sampler(m, EosVocab(eos), use_graph=use_graph, eos_per_row=True)
  for (tok, lens), fr in zip(runs, free):
    # same sampler twice (graph and its static buffers reused), stop on EOS
    st = s.generate(tok, lens, steps, end_sampling_at_eos_token=True)
    want = _expected_with_eos(fr, eos, 0)
    assert torch.equal(st.tokens_buffer.cpu(), want)
    hit = (fr == eos).any(dim=1)
    assert torch.equal(st.done.cpu(), hit)
  # without EOS stopping the same sampler reproduces the free run
  st = s.generate(*runs[0], steps, end_sampling_at_eos_token=False)
  assert torch.equal(st.tokens_buffer.cpu(), free[0])


def test_eos_all_rows_finish_early(dev):
  """Every row emits EOS at its first token: the loop ends long before
  `steps` and every later column is pad."""
  cfg = small_config(vocab=64, window=32)
  m, _ = make_model(dev, cfg, seed=32)
  tok = torch.full((3, 6), 5, dtype=torch.int32)
  lens = torch.full((3,), 6, dtype=torch.int32)
  first = cadence.Sampler(m, MockVocab(), use_graph=False).generate(
      tok, lens, 2).tokens_buffer.cpu()[:, 0]
  assert bool((first == first[0]).all())       # identical rows
  s = cadence.Sampler(m, EosVocab(int(first[0])), use_graph=True,
                      eos_per_row=True)
  st = s.generate(tok, lens, 64, end_sampling_at_eos_token=True)
  buf = st.tokens_buffer.cpu()
  assert torch.equal(buf[:, 0], first)
  assert bool((buf[:, 1:] == 0).all())
  assert int(st.step) < 64                     # stopped early
  assert bool(st.done.all())


@pytest.mark.parametrize("use_graph", [True, False])
def test_eos_reference_semantics(dev, use_graph):
  """Default mode = the reference loop: B > 1 never stops or pads; B = 1
  stops after a decode step emits EOS but not on the first token."""
  cfg = small_config(vocab=64, window=32)
  m, _ = make_model(dev, cfg, seed=34)
  steps = 40
  g = torch.Generator().manual_seed(5)
  tok = torch.randint(3, cfg.vocab_size, (3, 13), generator=g, dtype=torch.int32)
  lens = torch.full((3,), 13, dtype=torch.int32)
  free = cadence.Sampler(m, MockVocab(), use_graph=False).generate(
      tok, lens, steps).tokens_buffer.cpu()
  # an EOS every row emits somewhere after column 0: the batch still runs on
  eos = int(torch.mode(free[:, 1:].flatten()).values)
  s = cadence.Sampler(m, EosVocab(eos), use_graph=use_graph)
  st = s.generate(tok, lens, steps, end_sampling_at_eos_token=True)
  assert torch.equal(st.tokens_buffer.cpu(), free)
  assert not bool(st.done.any())
  # B = 1: each row alone, EOS = a token it emits after column 0
  for r in range(3):
    fr = cadence.Sampler(m, MockVocab(), use_graph=False).generate(
        tok[r:r + 1], lens[:1], steps).tokens_buffer.cpu()
    e = int(fr[0, steps // 2])
    s1 = cadence.Sampler(m, EosVocab(e), use_graph=use_graph)
    st = s1.generate(tok[r:r + 1], lens[:1], steps, end_sampling_at_eos_token=True)
    assert torch.equal(st.tokens_buffer.cpu(), _reference_loop(fr, e, 0)), (r, e)
    if r == 0:
      # the FIRST token as EOS: the reference does not stop on it
      e0 = int(fr[0, 0])
      s0 = cadence.Sampler(m, EosVocab(e0), use_graph=use_graph)
      st = s0.generate(tok[:1], lens[:1], steps, end_sampling_at_eos_token=True)
      assert torch.equal(st.tokens_buffer.cpu(), _reference_loop(fr, e0, 0))


def test_categorical_sampling(dev):
  """greedy_sampling=False: the first cached step and the loop both sample
  from logits (the first step used to receive logits=None)."""
  cfg = small_config(vocab=64, window=32)
  m, _ = make_model(dev, cfg, seed=33)
  with torch.no_grad():      # near-flat logits so samples differ from argmax
    m.embedder.input_embedding.mul_(0.01)
  g = torch.Generator().manual_seed(3)
  tok = torch.randint(3, cfg.vocab_size, (2, 9), generator=g, dtype=torch.int32)
  lens = torch.full((2,), 9, dtype=torch.int32)
  s = cadence.Sampler(m, MockVocab(), greedy_sampling=False)
  torch.manual_seed(123)
  a = s.generate(tok, lens, 12).tokens_buffer.cpu()
  torch.manual_seed(123)
  b = s.generate(tok, lens, 12).tokens_buffer.cpu()
  assert a.shape == (2, 12) and torch.equal(a, b)
  assert bool(((a >= 0) & (a < cfg.vocab_size)).all())
  torch.manual_seed(124)
  c = s.generate(tok, lens, 12, return_logits=True)
  assert c.logits_buffer.shape == (2, 12, 64)
  greedy = cadence.Sampler(m, MockVocab()).generate(tok, lens, 12).tokens_buffer
  assert not torch.equal(a, greedy.cpu())
  out = s(["Hello ! How are you?"], 5)
  assert out.tokens[0].shape == (5,)
