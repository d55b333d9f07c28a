"""Parity at the headline batch: the bench's B = 32 micro-batch path.

The full-size fixtures (tests/golden/make_golden_full.py) hold B <= 2, and
at B <= 2 the model takes other kernels than the bench does (the T-chunked
scan, split-K prefill GEMMs).  Here the same fixture samples are placed in a
batch of 32 -- at rows 0 and 31, with hashed filler samples between them --
so the prefill runs the kernels the headline runs (the fused RG-LRU gates +
scan `rglru_scan_fused_kernel`, non-split `gemm_big_kernel` at M = 32 L, the
MQA prefill attention over 32 sequences) and the decode runs the B = 32 hipGraph step.
Rows 0 and 31 are held to the bars of tests/test_full_size_gpu.py:

  * the prefill's last-position logits (final norm of the B = 32 prefill,
    then the logits GEMM on those rows);
  * teacher-forced decode logits (prefill on tokens[:, :-1], the cached step
    on the last prompt token, then the oracle's greedy tokens fed back;
    filler rows feed back their own argmax), examples/cadence_sampler.py:
    185-298 per row, i.e. the reference's B = 1 semantics
    (recurrentgemma/torch/griffin.py:171-172) row by row;
  * the graph sampler's tokens (Sampler.generate, exactly as bench.py calls
    it) equal the oracle's greedy tokens (up to the first step the oracle
    itself decides within a 0.2-logit margin).

Batches: bench224 (224 px, the bench's per-sample workload), c4 (336 px),
c2 (text-only, T = 2048).
"""

import json
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import hashinit as H  # noqa: E402
import make_golden_full as MG  # noqa: E402

import cadence  # noqa: E402
from cadence import _lib, ops  # noqa: E402
from test_full_size_gpu import _Vocab, _build, _check_row, _check_tokens, _fixture  # noqa: E402

pytestmark = pytest.mark.gpu
B = 32
ROWS = (0, B - 1)   # where the fixture samples go


def _batch(name, f, dev):
  """(tokens [B, T] int32 on dev, pixels [B, 3, S, S] or None, fixture row of
  ROWS[k]): fixture samples at rows 0 and 31, hashed fillers between."""
  size, b, t, _, seed = MG.CONFIGS[name]
  cfg = MG.griffin_config()
  tok = H.hash_tokens(B, t, cfg.vocab_size, seed * 7 + 91)
  src = [0, min(1, b - 1)]
  for r, j in zip(ROWS, src):
    tok[r] = f["tokens"][j]
  px = None
  if size is not None:
    px = H.hash_pixels(B, size, seed * 7 + 92, dev)
    fx = H.hash_pixels(b, size, seed * 7 + 2, dev)
    for r, j in zip(ROWS, src):
      px[r] = fx[j]
  return tok.to(dev), px, src


def _plan(L):
  """The kernels a B = 32 prefill of L tokens takes (the host-side plan
  queries of the C ABI): the fused RG-LRU gates + scan (the 2B preset: 10
  heads of 256 channels; x the conv output rows, the y gate a column slice
  of the packed [y | x] rows), the sequential scan where it is not taken (no
  chunk workspace), and the non-split big GEMM for the gated MLP and the
  recurrent projections."""
  lib = _lib.load()
  M = B * L
  aligned = 1 << 12          # host-only query: any 16-B aligned address
  assert lib.cadence_rglru_scan_plan(aligned, 2560, aligned, 5120, 2560, B, L, 10,
                                     256) == 1, "fused RG-LRU gates + scan"
  assert lib.cadence_rnn_scan_workspace_bytes(B, L, 2560) == 0, "chunked scan"
  for n, k in ((2 * 7680, 2560), (2 * 2560, 2560), (2560, 7680)):
    assert lib.cadence_gemm_big_splits(M, n, k, 1) == 1, f"split-K at {M}x{n}x{k}"


@pytest.mark.parametrize("name", ["bench224", "c4", "c2"])
def test_headline_batch_parity(dev, name):
  f, meta = _fixture(name)
  size, _, t, steps, _ = MG.CONFIGS[name]
  m, cfg, vis = _build(name, dev, f, meta)
  tok, px, src = _batch(name, f, dev)
  n_vis = 0 if vis is None else vis.n_visual_tokens
  _plan(n_vis + t)
  _plan(n_vis + t - 1)
  pos = torch.arange(t, dtype=torch.int32, device=dev)[None].repeat(B, 1)
  cap = float(cfg.logits_soft_cap or 0.0)
  report, bad = {}, []
  with torch.no_grad():
    # prefill over [image | prompt] at B = 32, then the last position's
    # logits (the full [B, L, V] logits of C2 would be 33 GB)
    x, p2, L = m.embed_inputs(tok, pos, images=px)
    _, xn, _ = m.run_blocks(x, p2, B, L, None, False, final_norm=True)
    last = xn.view(B, L, -1)[:, -1].contiguous()
    logits = ops.gemm_logits(last, m.embedder.input_embedding, cap)
    del x, xn
    for r, j in zip(ROWS, src):
      report[f"prefill[{r}]"] = _check_row(logits[r], f, j, 0,
                                           f"{name} B=32 prefill row {r}", bad)
    # teacher-forced decode at B = 32 (eager steps; the graph replays the
    # same launches, tests/test_model_gpu.py checks graph == eager)
    _, cache = m(tok[:, :-1], pos[:, :-1], images=px, return_logits=False,
                 image_splice=px is not None)
    gt = f["greedy_tokens"].to(dev)
    cur, p = tok[:, -1:].clone(), pos[:, -1:]
    for s in range(steps):
      nxt, lg, cache = m.next_token(cur, p, cache, return_logits=True)
      for r, j in zip(ROWS, src):
        report[f"step{s}[{r}]"] = _check_row(lg[r], f, j, 1 + s,
                                             f"{name} B=32 decode step {s} row {r}",
                                             bad)
      cur = nxt.to(torch.int32)[:, None].clone()
      for r, j in zip(ROWS, src):
        cur[r, 0] = gt[j, s]
      p = p + 1
    del cache
  # the bench's own call: Sampler.generate with the captured decode graph
  st = cadence.Sampler(m, _Vocab()).generate(
      tok, torch.full((B,), t, dtype=torch.int32), steps, images=px)
  got = st.tokens_buffer.cpu()
  for r, j in zip(ROWS, src):
    report[f"sampler[{r}]"] = _check_tokens(got[r], f, j, f"{name} B=32 row {r}", bad)
  print(name, "B=32", json.dumps(report), flush=True)
  assert not bad, "\n".join(bad)
