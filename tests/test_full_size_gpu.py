"""Full-size parity: every BASELINE.json configuration's real model on the GPU.

The RecurrentGemma-2B preset (26 blocks, width 2560, vocab 256000) and, for
the image configurations, the full 23-block DINOv2-L/14-reg4 + SigLIP-
so400m/14 towers + projector, with the fixture weights rebuilt on the
device from tests/golden/hashinit.py (bit-exact: every tensor's probe
values are compared exactly) and checked against the CPU oracle's outputs
committed by tests/golden/make_golden_full.py:

  c1        text-only, B=1, T=16, 8 decode steps   (BASELINE config 1's shape)
  c2        text-only, B=1, T=2048, 4 steps        (config 2's prompt length)
  c3        224 px, B=1, T=64, 8 steps             (config 3)
  bench224  224 px, B=2, T=64, 4 steps             (the bench workload per sample)
  c4        336 px, B=1, T=64, 4 steps             (config 4; ViT N = 581 / 576)
  p0        384 px, B=1, T=16, 4 steps             (the reference's own size, n_vis 729)

Bars: vision features rel-L2 <= 1e-2 against the fp32 towers
(bf16 MFMA, fp32 residual stream), projector rel-L2 <= 2e-2; logits of the
prefill forward's last position and of every teacher-forced decode step
(the oracle's greedy tokens fed back, examples/cadence_sampler.py:185-298),
on the oracle's top-256 + 4096 fixed vocabulary entries:
  * cosine >= 0.999 against the bf16 oracle;
  * accuracy against an fp32 run of the same op sequence (`logit_val_fp32`,
    make_golden_full.add_fp32): max-abs and rel-L2 of the HIP path's error
    at most 1.25x the bf16 oracle's own error (+0.02 / +0.005).  SURVEY's
    "max-abs <= 0.1 vs the reference" cannot be the bar: the reference's own
    bf16 arithmetic is 0.10-0.15 from fp32 on these logits (printed by
    make_golden_full.py), and two bf16 pipelines of that accuracy differ by
    up to twice that; so max-abs vs the bf16 oracle is capped at 0.25;
  * greedy token equal wherever the oracle's top-1/top-2 margin exceeds 0.2
    (else within the oracle's top 2);
the hipGraph sampler's tokens equal the oracle's greedy tokens.
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
  if c < COS:
    bad.append(f"{what}: cosine {c:.6f}")
  if err > MAX_ABS:
    bad.append(f"{what}: max-abs {err:.4f} vs the bf16 oracle at want "
               f"{float(want[w]):.4f} got {float(sub[w]):.4f}")
  ours = float((sub - exact).abs().max())
  ref = float((want - exact).abs().max())
  ours_l2, ref_l2 = rel_l2(sub, exact), rel_l2(want, exact)
  if ours > ACC * ref + 0.02:
    bad.append(f"{what}: max-abs vs fp32 {ours:.4f}, bf16 oracle's own {ref:.4f}")
  if ours_l2 > ACC * ref_l2 + 0.005:
    bad.append(f"{what}: rel-L2 vs fp32 {ours_l2:.5f}, bf16 oracle's own "
               f"{ref_l2:.5f}")
  top2 = idx[torch.topk(want, 2).indices]
  am = int(got.float().argmax())
  if float(f["logit_margin"][i, j]) > MARGIN:
    if am != int(top2[0]):
      bad.append(f"{what}: argmax {am} vs {int(top2[0])}")
  elif am not in top2.tolist():
    bad.append(f"{what}: argmax {am} not in oracle top-2")
  return {"cos": round(c, 6), "max_abs_vs_oracle": round(err, 4),
          "max_abs_vs_fp32": round(ours, 4), "oracle_max_abs_vs_fp32": round(ref, 4),
          "rel_l2_vs_fp32": round(ours_l2, 5), "oracle_rel_l2_vs_fp32": round(ref_l2, 5)}


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
  ok = bool((f["logit_margin"][:, 1:] > MARGIN).all())
  st = cadence.Sampler(m, _Vocab()).generate(
      tok, torch.full((b,), t, dtype=torch.int32), steps, images=px)
  if ok and not torch.equal(st.tokens_buffer.cpu(), f["greedy_tokens"]):
    bad.append(f"{name}: sampler tokens {st.tokens_buffer.tolist()}")
  print(name, json.dumps(report), flush=True)
  assert not bad, "\n".join(bad)
