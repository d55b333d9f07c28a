"""Weight-seed search for __graft_entry__.smoke (TEST INFRASTRUCTURE).

Runs the smoke's oracle side only (CPU): for each seed, the greedy
continuation of both samples and the oracle's top-1 / top-2 margin per step.
A seed qualifies when every sample's continuation has >= 3 distinct tokens
and its first MIN_DECIDED steps are decided by the margin (so the GPU must
match them exactly).

    python tools/smoke_seed_search.py STEPS MIN_DECIDED SEED [SEED ...]
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cadence-gemma_amd"), os.path.join(ROOT, "tests", "golden")]


def main():
  import torch
  import __graft_entry__ as G
  from oracle import griffin_ref as R
  import hashinit as H
  cfg, vis = G.smoke_configs()
  steps, need = int(sys.argv[1]), int(sys.argv[2])
  import cadence
  b, t = 2, 8
  with torch.no_grad():
    m = cadence.Griffin(cfg, device="meta", dtype=torch.bfloat16, vision=vis)
  shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
  for seed in [int(s) for s in sys.argv[3:]]:
    p = H.hash_params(shapes, seed, cfg.num_layers)
    px = H.hash_pixels(b, 28, seed * 7 + 2)
    tok = H.hash_tokens(b, t, cfg.vocab_size, seed * 7 + 1)
    want_tok, want_logits = R.greedy_sample(p, cfg, tok.long(), steps, pixels=px, vcfg=vis)
    decided, distinct = [], []
    for i in range(b):
      n = 0
      while n < steps:
        top = torch.topk(want_logits[i, n].float(), 2)
        if float(top.values[0] - top.values[1]) <= G.SMOKE_MARGIN:
          break
        n += 1
      decided.append(n)
      distinct.append(len(set(want_tok[i].tolist())))
    ok = min(decided) >= need and min(distinct) >= 3
    print(f"seed {seed}: tokens {want_tok.tolist()} decided {decided} distinct {distinct}"
          f"{'  <== ok' if ok else ''}", flush=True)


if __name__ == "__main__":
  main()
