"""Full-size golden fixtures: every BASELINE.json configuration's real model.

TEST INFRASTRUCTURE.  The CPU oracle (oracle/griffin_ref.py) runs the
RecurrentGemma-2B preset (26 blocks, width 2560, vocab 256000) and, for the
multimodal configurations, the full DINOv2-L/14-reg4 + SigLIP-so400m/14
towers (23 blocks each, fp32, as the reference's timm towers) + projector,
at each configuration's image size.  Weights, pixels and prompts come from
the device-independent hash of tests/golden/hashinit.py, so the GPU test
(tests/test_full_size_gpu.py) rebuilds the identical model on the device
and checks it bit-exactly against the probes stored here.

Stored per configuration (tests/golden/full_<name>.safetensors):
  * prompt tokens;
  * for images: 24 feature rows per sample (fp32) and the same projector
    output rows (the vision tower at full depth, rel-L2 bar 1e-2);
  * logits: the prefill forward's last position, then the greedy decode's
    per-step logits (examples/cadence_sampler.py:185-298: prefill on
    tokens[:, :-1], cached step on the last prompt token, decode), each on
    the oracle's top-256 entries + 4096 fixed hashed vocabulary entries,
    with the oracle's top-1 / top-2 margin;
  * the oracle's greedy tokens (the GPU test teacher-forces them);
  * weight checksums (float64 sums) and 16 probe values per tensor.

    python tests/golden/make_golden_full.py [name ...]
"""

from __future__ import annotations

import json
import os
import sys
import time

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for _p in (os.path.join(ROOT, "cadence-gemma_amd"), ROOT, HERE):
  if _p not in sys.path:
    sys.path.insert(0, _p)

import hashinit as H  # noqa: E402
from cadence import common  # noqa: E402

BF = torch.bfloat16
N_RANDOM_IDX = 4096
N_TOP_IDX = 256
N_FEATURE_ROWS = 24

# name -> (image size or None, batch, prompt length, decode steps, weight seed)
# c1..c4 follow BASELINE.json's configs (c1 is the CPU plumbing config's
# shape, here run on the GPU against the oracle); bench224 is the bench's
# per-sample workload (224 px, 64-token prompt) at batch 2; p0 is 384 px,
# the only size the reference itself accepts (griffin.py:186-191).
CONFIGS = {
    "c1": (None, 1, 16, 8, 101),
    "c2": (None, 1, 2048, 8, 132),
    "c3": (224, 1, 64, 8, 203),
    "bench224": (224, 2, 64, 8, 287),
    "c4": (336, 1, 64, 8, 313),
    "p0": (384, 1, 16, 8, 440),
}


def griffin_config():
  return common.GriffinConfig.from_preset(common.Preset.RECURRENT_GEMMA_2B_V1)


def vision_config(size):
  return None if size is None else common.VisionConfig(image_size=size)


def state_shapes(cfg, vis):
  import cadence
  m = cadence.Griffin(cfg, device="meta", dtype=BF, vision=vis)
  return {k: tuple(v.shape) for k, v in m.state_dict().items()}


def params(name, device="cpu"):
  size, _, _, _, seed = CONFIGS[name]
  cfg, vis = griffin_config(), vision_config(size)
  return H.hash_params(state_shapes(cfg, vis), seed, cfg.num_layers, device)


def inputs(name, device="cpu"):
  size, b, t, _, seed = CONFIGS[name]
  cfg = griffin_config()
  tok = H.hash_tokens(b, t, cfg.vocab_size, seed * 7 + 1)
  px = None if size is None else H.hash_pixels(b, size, seed * 7 + 2, device)
  return tok, px


def feature_rows(n_vis):
  return torch.linspace(0, n_vis - 1, N_FEATURE_ROWS).round().long()


def random_vocab_idx(vocab):
  u = H.hash_uniform(N_RANDOM_IDX, 77, "cpu").double()
  return torch.unique((u * vocab).long())


def logit_subset(row, rnd):
  """row [V] fp32 -> (idx [K] int32, val [K] fp32, top1 - top2)."""
  top = torch.topk(row, N_TOP_IDX)
  idx = torch.cat([top.indices, rnd])
  idx = torch.unique(idx)
  k = N_TOP_IDX + N_RANDOM_IDX
  if idx.numel() < k:        # pad with entries not yet chosen (fixed order)
    extra = torch.tensor([i for i in range(2 * k) if i not in set(idx.tolist())])
    idx = torch.cat([idx, extra[:k - idx.numel()]]).sort().values
  idx = idx[:k]
  margin = float(top.values[0] - top.values[1])
  return idx.to(torch.int32), row[idx].float(), margin


def forced_rows(p, cfg, tok, gtok, img, R):
  """Oracle logits [B, 1 + S, V]: the prefill forward's last position, then
  prefill on tokens[:, :-1], the cached step on the last prompt token and
  the given tokens fed back (teacher forcing)."""
  b, t = tok.shape
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  last, _ = R.griffin_forward(p, cfg, tok, pos, image_tokens=img,
                              last_only=True)
  _, cache = R.griffin_forward(p, cfg, tok[:, :-1], pos[:, :-1],
                               image_tokens=img, return_logits=False)
  rows = [last[:, 0]]
  cur, pp = tok[:, -1:], pos[:, -1:]
  for s in range(gtok.shape[1]):
    lg, cache = R.griffin_forward(p, cfg, cur.to(torch.int32), pp, cache=cache)
    rows.append(lg[:, 0])
    cur, pp = gtok[:, s:s + 1], pp + 1
  return torch.stack(rows, 1)


def projector_fp32(feats, p):
  """projector/mlp.py:13-31 without the bf16 casts (fp32 reference run)."""
  import torch.nn.functional as F
  x = feats.float()
  idx = sorted({int(k.split(".")[2]) for k in p if k.startswith("projector.proj.")})
  for j, li in enumerate(idx):
    x = F.linear(x, p[f"projector.proj.{li}.weight"].float(),
                 p[f"projector.proj.{li}.bias"].float())
    if j < len(idx) - 1:
      x = F.gelu(x)
  return x


def add_fp32(name, p=None):
  """The same oracle op sequence with every weight and activation in fp32
  (teacher-forced with the bf16 oracle's greedy tokens): how far the
  reference's own bf16 arithmetic is from an fp32 computation, stored at
  the fixture's logit indices as `logit_val_fp32`, and the vision features
  as `features_fp32_check` (the towers already run in fp32)."""
  from oracle import griffin_ref as R
  from safetensors import safe_open
  from safetensors.torch import load_file
  size, b, t, steps, seed = CONFIGS[name]
  cfg, vis = griffin_config(), vision_config(size)
  path = os.path.join(HERE, f"full_{name}.safetensors")
  with safe_open(path, "pt") as fh:
    meta = fh.metadata()
  out = load_file(path)
  t0 = time.time()
  if p is None:
    p = params(name)
  p32 = {k: v.float() for k, v in p.items()}
  del p
  tok, px = inputs(name)
  img = None
  if vis is not None:
    img = projector_fp32(R.vision_encoder(px, p32, vis), p32)
  rows = forced_rows(p32, cfg, tok.long(), out["greedy_tokens"].long(), img, R)
  idx = out["logit_idx"].long()
  out["logit_val_fp32"] = torch.gather(rows.float(), 2, idx).contiguous()
  save_file({k: v.contiguous() for k, v in out.items()}, path, metadata=meta)
  d = (out["logit_val"] - out["logit_val_fp32"]).abs()
  print(f"{name} fp32: {time.time() - t0:.1f} s; bf16 oracle vs fp32 max-abs "
        f"per row {d.amax(-1).tolist()}", flush=True)


def make(name):
  from oracle import griffin_ref as R
  size, b, t, steps, seed = CONFIGS[name]
  cfg, vis = griffin_config(), vision_config(size)
  t0 = time.time()
  p = params(name)
  tok, px = inputs(name)
  print(f"{name}: weights {time.time() - t0:.1f} s", flush=True)
  out = {"tokens": tok}
  img = None
  if vis is not None:
    feats = R.vision_encoder(px, p, vis)
    img = R.projector(feats, p)
    rows = feature_rows(vis.n_visual_tokens)
    out["feature_rows"] = rows.to(torch.int32)
    out["features"] = feats[:, rows].float().contiguous()
    out["image_tokens"] = img[:, rows].float().contiguous()
  pos = torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  last, _ = R.griffin_forward(p, cfg, tok.long(), pos, image_tokens=img,
                              last_only=True)
  gtok, glog = R.greedy_sample(p, cfg, tok.long(), steps, pixels=px, vcfg=vis)
  rnd = random_vocab_idx(cfg.vocab_size)
  idx, val, margin = [], [], []
  for i in range(b):
    rows = [last[i, 0].float()] + [glog[i, s].float() for s in range(steps)]
    r = [logit_subset(x, rnd) for x in rows]
    idx.append(torch.stack([x[0] for x in r]))
    val.append(torch.stack([x[1] for x in r]))
    margin.append(torch.tensor([x[2] for x in r]))
  out["logit_idx"] = torch.stack(idx)          # [B, 1 + S, K]
  out["logit_val"] = torch.stack(val)
  out["logit_margin"] = torch.stack(margin)    # [B, 1 + S]
  out["greedy_tokens"] = gtok.to(torch.int32)
  out["param_sums"] = H.checksums(p)
  out["param_probes"] = H.probes(p)
  meta = {"config": json.dumps({"name": name, "image_size": size, "batch": b,
                                "prompt": t, "steps": steps, "seed": seed}),
          "param_keys": ",".join(sorted(p))}
  path = os.path.join(HERE, f"full_{name}.safetensors")
  save_file({k: v.contiguous() for k, v in out.items()}, path, metadata=meta)
  print(f"{name}: {time.time() - t0:.1f} s, {os.path.getsize(path)} bytes, "
        f"greedy {gtok.tolist()}, margins {out['logit_margin'].tolist()}",
        flush=True)
  add_fp32(name, p)


def main():
  torch.set_num_threads(min(8, os.cpu_count() or 1))
  args = sys.argv[1:]
  if args and args[0] == "--fp32-only":        # add the fp32 rows only
    for name in (args[1:] or list(CONFIGS)):
      add_fp32(name)
    return
  for name in (args or list(CONFIGS)):
    make(name)


if __name__ == "__main__":
  main()
