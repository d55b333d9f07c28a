"""Full-size parity: every BASELINE.json configuration's real model on the GPU.

The RecurrentGemma-2B preset (26 blocks, width 2560, vocab 256000) and, for
the image configurations, the full 23-block DINOv2-L/14-reg4 + SigLIP-
so400m/14 towers + projector, with the fixture weights rebuilt on the
device from tests/golden/hashinit.py (bit-exact: every tensor's probe
values are compared exactly) and checked against the CPU oracle's outputs
committed by tests/golden/make_golden_full.py:

  c1        text-only, B=1, T=16, 8 decode steps   (BASELINE config 1's shape)
  c2        text-only, B=1, T=2048, 8 steps        (config 2's prompt length)
  c3        224 px, B=1, T=64, 8 steps             (config 3)
  bench224  224 px, B=2, T=64, 8 steps             (the bench workload per sample)
  c4        336 px, B=1, T=64, 8 steps             (config 4; ViT N = 581 / 576)
  p0        384 px, B=1, T=16, 8 steps             (the reference's own size, n_vis 729)

The fixture weights (hashinit.param_spec) put the residual projections at
5 / sqrt(fan_in) and the tied embedding at 1.5 / sqrt(D), so the blocks,
not the input token's own embedding, decide the logits: greedy
continuations vary (>= 3 distinct tokens per row, checked on the CPU by
tests/test_full_fixtures_cpu.py) with top-1 / top-2 margins of a fraction of
a logit to a few logits, and the teacher-forced decode feeds changing tokens.

Bars: vision features rel-L2 <= 1e-2 against the fp32 towers
(bf16 MFMA, fp32 residual stream), projector rel-L2 <= 2e-2; logits of the
prefill forward's last position and of every teacher-forced decode step
(the oracle's greedy tokens fed back, examples/cadence_sampler.py:185-298),
on the oracle's top-256 + 4096 fixed vocabulary entries:
  * against the bf16 oracle: cosine >= 0.999 -- or, where the oracle's own
    cosine to the fp32 run is 1 - e with 2e > 0.001, >= 1 - 2e (two bf16
    pipelines each e from fp32); max-abs at most max(0.25, 2x the oracle's
    own max-abs distance from fp32);
  * accuracy against an fp32 run of the same op sequence (`logit_val_fp32`,
    make_golden_full.add_fp32): max-abs and rel-L2 of the HIP path's error
    at most 1.25x the bf16 oracle's own error (+0.02 / +0.005).  SURVEY's
    "max-abs <= 0.1 vs the reference" cannot be the bar: the reference's own
    bf16 arithmetic is 0.25-0.7 from fp32 on these logits (printed by
    make_golden_full.py), and two bf16 pipelines of that accuracy differ by
    up to twice that;
  * greedy token equal wherever the oracle's top-1/top-2 margin exceeds the
    larger of 0.2 and 1.5x the oracle's own max-abs distance from fp32 on
    that row (else within the oracle's top 2);
the hipGraph sampler's tokens equal the oracle's greedy tokens up to the
first step whose margin is within that bar (there: one of the oracle's top
2; the continuations may part after it).
"""

import json
import os
import sys

import pytest
import torch
from safetensors import safe_open
from safetensors.torch import load_file

from conftest import cosine, rel_l2

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import hashinit as H  # noqa: E402
import make_golden_full as MG  # noqa: E402

import cadence  # noqa: E402

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
MAX_ABS = 0.25
COS = 0.999
ACC = 1.25
MARGIN = 0.2
# every fixture row's sampler continuation is compared for at least this
# many steps (the fixture seeds are chosen so the oracle's first decode steps
# are margin-decided: tests/golden/seed_search.py)
MIN_STEPS_COMPARED = 3
# per-row reports (cosine, max-abs, rel-L2 vs fp32, steps compared) land
# here on every run, pass or fail, for the evidence under profiles/
REPORT_DIR = os.environ.get("CADENCE_PARITY_REPORT_DIR", os.path.join(
    os.path.dirname(HERE), "gpurun_out", "parity"))


class _Vocab:
  def pad_id(self):
    return 0

  def bos_id(self):
    return 2

  def eos_id(self):
    return 1


def _fixture(name):
  path = os.path.join(HERE, "golden", f"full_{name}.safetensors")
  with safe_open(path, "pt") as f:
    meta = f.metadata()
  return load_file(path), meta


def _build(name, dev, f, meta):
  size, _, _, _, seed = MG.CONFIGS[name]
  cfg, vis = MG.griffin_config(), MG.vision_config(size)
  with torch.no_grad():
    m = cadence.Griffin(cfg, device=dev, dtype=BF, vision=vis)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert ",".join(sorted(shapes)) == meta["param_keys"]
    p = H.hash_params(shapes, seed, cfg.num_layers, device=dev)
    probes = H.probes(p)
    assert torch.equal(probes, f["param_probes"]), "device weights differ"
    torch.testing.assert_close(H.checksums(p), f["param_sums"], rtol=1e-9,
                               atol=1e-6)
    m.load_state_dict(p)
    del p
  m.eval()
  return m, cfg, vis


def _margin_bar(f, i, j):
  """The top-1 / top-2 margin above which the oracle's choice is decided by
  the reference arithmetic rather than its bf16 noise: MARGIN, or 1.5x the
  oracle's own max-abs distance from the fp32 run on that row."""
  d = float((f["logit_val"][i, j] - f["logit_val_fp32"][i, j]).abs().max())
  return max(MARGIN, 1.5 * d)


def _check_row(got, f, i, j, what, bad):
  """got: [V] logits of sample i, fixture row j (0 = prefill last position,
  1 + s = decode step s).  Violations go to `bad` (reported together)."""
  idx = f["logit_idx"][i, j].long()
  want = f["logit_val"][i, j]
  exact = f["logit_val_fp32"][i, j]
  sub = got.float().cpu()[idx]
  c = cosine(sub, want)
  d = (sub - want).abs()
  err = float(d.max())
  w = int(d.argmax())
  # two pipelines each (1 - c_ref) from fp32 in cosine are up to about
  # twice that apart: the bar is COS unless the oracle itself is further
  cos_bar = min(COS, 1.0 - 2.0 * (1.0 - cosine(want, exact)))
  if c < cos_bar:
    bad.append(f"{what}: cosine {c:.6f} (bar {cos_bar:.6f})")
  ours = float((sub - exact).abs().max())
  ref = float((want - exact).abs().max())
  # two bf16 pipelines each `ref` from fp32 differ by up to about twice it
  if err > max(MAX_ABS, 2.0 * ref):
    bad.append(f"{what}: max-abs {err:.4f} vs the bf16 oracle (bar "
               f"{max(MAX_ABS, 2.0 * ref):.4f}) at want {float(want[w]):.4f} got "
               f"{float(sub[w]):.4f}")
  ours_l2, ref_l2 = rel_l2(sub, exact), rel_l2(want, exact)
  if ours > ACC * ref + 0.02:
    bad.append(f"{what}: max-abs vs fp32 {ours:.4f}, bf16 oracle's own {ref:.4f}")
  if ours_l2 > ACC * ref_l2 + 0.005:
    bad.append(f"{what}: rel-L2 vs fp32 {ours_l2:.5f}, bf16 oracle's own "
               f"{ref_l2:.5f}")
  top2 = idx[torch.topk(want, 2).indices]
  am = int(got.float().argmax())
  if float(f["logit_margin"][i, j]) > _margin_bar(f, i, j):
    if am != int(top2[0]):
      bad.append(f"{what}: argmax {am} vs {int(top2[0])}")
  elif am not in top2.tolist():
    bad.append(f"{what}: argmax {am} not in oracle top-2")
  return {"cos": round(c, 6), "cos_bar": round(cos_bar, 6),
          "max_abs_vs_oracle": round(err, 4),
          "max_abs_vs_fp32": round(ours, 4), "oracle_max_abs_vs_fp32": round(ref, 4),
          "rel_l2_vs_fp32": round(ours_l2, 5), "oracle_rel_l2_vs_fp32": round(ref_l2, 5)}


def _check_tokens(got, f, i, what, bad):
  """A sampler's greedy tokens `got` [S] against the oracle's for fixture
  sample i, step by step: equal while the oracle's top-1 / top-2 margin
  exceeds _margin_bar; at a step whose margin does not, the token must be one of
  the oracle's top 2, and where it is the other one the two continuations
  may legitimately part (the later steps are not compared).  Returns the
  number of steps compared."""
  want = f["greedy_tokens"][i]
  for s in range(want.numel()):
    g, w = int(got[s]), int(want[s])
    if float(f["logit_margin"][i, 1 + s]) > _margin_bar(f, i, 1 + s):
      if g != w:
        bad.append(f"{what}: sampler token {s} is {g}, oracle {w} "
                   f"(tokens {got.tolist()} vs {want.tolist()})")
        return s
      continue
    idx = f["logit_idx"][i, 1 + s].long()
    top2 = idx[torch.topk(f["logit_val"][i, 1 + s], 2).indices].tolist()
    if g not in top2:
      bad.append(f"{what}: sampler token {s} is {g}, not in the oracle's top 2 {top2}")
    if g != w:
      return s + 1
  return want.numel()


@pytest.mark.parametrize("name", list(MG.CONFIGS))
def test_full_size_parity(dev, name):
  f, meta = _fixture(name)
  size, b, t, steps, seed = MG.CONFIGS[name]
  m, cfg, vis = _build(name, dev, f, meta)
  tok = f["tokens"].to(dev)
  assert tok.shape == (b, t)
  px = None if size is None else H.hash_pixels(b, size, seed * 7 + 2, dev)
  pos = torch.arange(t, dtype=torch.int32, device=dev)[None].repeat(b, 1)
  report, bad = {}, []
  with torch.no_grad():
    if vis is not None:
      feats = m.vis_encoder.encode(px)
      assert feats.shape == (b, vis.n_visual_tokens, vis.feature_width)
      rows = f["feature_rows"].long().to(dev)
      for i in range(b):
        e = rel_l2(feats[i, rows], f["features"][i])
        if e > 1e-2:
          bad.append(f"{name}: vision features rel-L2 {e:.5f}")
        report[f"features_rel_l2[{i}]"] = round(e, 6)
      e = rel_l2(m.projector(feats)[:, rows], f["image_tokens"])
      if e > 2e-2:
        bad.append(f"{name}: projector rel-L2 {e:.5f}")
      report["image_tokens_rel_l2"] = round(e, 6)
    # prefill forward over [image | prompt]: last position
    logits, _ = m(tok, pos, images=px)
    for i in range(b):
      report[f"prefill[{i}]"] = _check_row(logits[i, -1], f, i, 0,
                                           f"{name} prefill row {i}", bad)
    del logits
    # teacher-forced decode: prefill tokens[:, :-1], cached step on the last
    # prompt token, then the oracle's greedy tokens fed back one by one
    _, cache = m(tok[:, :-1], pos[:, :-1], images=px, return_logits=False)
    gt = f["greedy_tokens"].to(dev)
    cur, p = tok[:, -1:], pos[:, -1:]
    for s in range(steps):
      nxt, lg, cache = m.next_token(cur, p, cache, return_logits=True)
      for i in range(b):
        report[f"step{s}[{i}]"] = _check_row(lg[i], f, i, 1 + s,
                                             f"{name} decode step {s} row {i}",
                                             bad)
      cur, p = gt[:, s:s + 1], p + 1
  # the graph-replayed sampler reproduces the oracle's greedy continuation
  st = cadence.Sampler(m, _Vocab()).generate(
      tok, torch.full((b,), t, dtype=torch.int32), steps, images=px)
  got = st.tokens_buffer.cpu()
  for i in range(b):
    n = _check_tokens(got[i], f, i, f"{name} row {i}", bad)
    if n < MIN_STEPS_COMPARED:
      bad.append(f"{name} row {i}: sampler tokens compared for {n} steps "
                 f"(floor {MIN_STEPS_COMPARED})")
    report[f"sampler[{i}]"] = {
        "steps_compared": n, "tokens": got[i].tolist(),
        "oracle_tokens": f["greedy_tokens"][i].tolist(),
        "distinct_oracle_tokens": len(set(f["greedy_tokens"][i].tolist()))}
  report["argmax_enforced_rows"] = sum(
      float(f["logit_margin"][i, j]) > _margin_bar(f, i, j)
      for i in range(b) for j in range(1 + steps))
  report["rows"] = b * (1 + steps)
  report["violations"] = bad
  print(name, json.dumps(report), flush=True)
  os.makedirs(REPORT_DIR, exist_ok=True)
  with open(os.path.join(REPORT_DIR, f"full_{name}.json"), "w") as fh:
    json.dump(report, fh, indent=1)
  assert not bad, "\n".join(bad)
