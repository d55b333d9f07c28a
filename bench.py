#!/usr/bin/env python
"""CadenceGemma multimodal prefill+decode benchmark on MI355X.

Metric (BASELINE.json): multimodal prefill+decode tokens/sec, Cadence-2B,
224 px, bs=32, 1 -> 8 MI355X.  One step = the global batch of 256 (image,
prompt) samples (strong scaling, k GPUs each run 256 / (32 k)
micro-batches of 32) through the whole hot path: dual ViT (DINOv2-L/14-reg4
+ SigLIP-so400m/14, 23 blocks each) -> projector -> Griffin-2B prefill on
[image | prompt[:-1]] -> cached step on the last prompt token -> 31 greedy
decode steps (hipGraph replay) per micro-batch, then one all-gather of the
generated tokens (RCCL on N > 1).  Tokens per step = 256 * (256+64+32).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU)
  python bench.py --config c2|c3|c4                      (the other configs)

Prints ONE JSON line on rank 0 (see the driver contract in the task).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "cadence-gemma_amd"), ROOT):
  if _p not in sys.path:
    sys.path.insert(0, _p)

import torch  # noqa: E402

import cadence  # noqa: E402
from cadence import common, distributed as D, ops  # noqa: E402

METRIC = ("multimodal prefill+decode tokens/sec, Cadence-2B 224px bs=32, "
          "1→8 MI355X")
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_BF16_PEAK_TFS = 2500.0    # dense bf16 MFMA spec

# Where a key's meaning changed between rounds (lines of different rounds are
# comparable only where the version matches).
DEFINITIONS = {
    "version": 6,
    "prefill_tokens_per_s": "aggregate over ranks since round 5 (per rank before)",
    "value (config c3)": "one request at a time since round 5 (two requests in "
                         "flight before; that rate is value_serving now)",
    "roofline_scan": "the RG-LRU scan kernel the workload runs since round 6 "
                     "(rglru_scan_fused_kernel at the headline shape); the "
                     "isolated rnn_scan_kernel figure is roofline_scan_isolated",
}


def scaling_inputs(world, gb, tok_per_step, ms_step, rank_ms, rank_prefill_ms,
                   prefill_tps):
  """The quantities a 1 -> N speed-up is computed from, on both the
  end-to-end value and the prefill rate: each rank's own wall time per step
  (its share gb / world of the global batch), the slowest of them (what
  `value` divides by), and each rank's timed prefill."""
  return {"world": world, "global_batch": gb, "samples_per_rank": gb // world,
          "tokens_per_step": tok_per_step,
          "end_to_end_ms_per_step": round(ms_step, 3),
          "end_to_end_ms_per_step_by_rank": [round(v, 3) for v in rank_ms],
          "prefill_ms_by_rank": [round(v, 3) for v in rank_prefill_ms],
          "prefill_tokens_per_s": round(prefill_tps, 1)}


class BenchVocab:
  """Synthetic token ids only; the Gemma tokenizer is not shipped."""

  def pad_id(self):
    return 0

  def bos_id(self):
    return 2

  def eos_id(self):
    return 1


# SURVEY §8d configurations (BASELINE.json configs 2-4); the default is the
# metric's workload (C5 shape at 224 px: global batch 256, micro-batch 32).
CONFIGS = {
    "bench": dict(image_size=224, batch=32, global_batch=256, prompt=64,
                  decode=32, text_only=False),
    "c2": dict(image_size=224, batch=32, global_batch=0, prompt=2048,
               decode=64, text_only=True),
    "c3": dict(image_size=224, batch=1, global_batch=0, prompt=64, decode=32,
               text_only=False),
    "c4": dict(image_size=336, batch=32, global_batch=0, prompt=64, decode=0,
               text_only=False),
}


def parse(argv=None):
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=5)
  ap.add_argument("--warmup", type=int, default=2)
  ap.add_argument("--config", choices=sorted(CONFIGS), default="bench")
  ap.add_argument("--batch", type=int, help="micro-batch (samples per launch "
                  "chain on one GPU)")
  ap.add_argument("--global-batch", type=int,
                  help="samples per step over all ranks (strong scaling); 0 = "
                  "batch x world (weak scaling)")
  ap.add_argument("--image-size", type=int)
  ap.add_argument("--prompt", type=int)
  ap.add_argument("--decode", type=int)
  ap.add_argument("--no-cpu-baseline", action="store_true")
  ap.add_argument("--cpu-decode-steps", type=int)
  ap.add_argument("--no-kernel-timing", action="store_true")
  ap.add_argument("--text-only", action="store_true", default=None,
                  help="C2-style text-only run (no vision tower)")
  ap.add_argument("--no-pipeline", action="store_true",
                  help="run the micro-batches back to back (generate per "
                  "micro-batch) instead of Sampler.generate_many's pipeline")
  ap.add_argument("--no-continuous", action="store_true",
                  help="lab A/B: join the pipeline lanes at the end of every "
                  "step (no overlap of step i + 1's first prefill with step "
                  "i's last decode; one micro-batch per rank then runs plain "
                  "Sampler.generate)")
  ap.add_argument("--split-single", action="store_true",
                  help="lab: a rank whose share is one micro-batch runs it as "
                  "two pipelined halves (generate_many) instead of whole; "
                  "measured slower (profiles/r04c_n8_load_*: 135.7 vs 103.6 "
                  "ms for 32 samples -- a decode step streams every weight "
                  "whatever its row count, so two halves stream them twice)")
  ap.add_argument("--gemm-engine", type=int, default=None,
                  help="lab A/B: prefill GEMM engine plan (cadence_gemm_set_engine)")
  ap.add_argument("--serving-pass", action="store_true", default=None,
                  help="after the headline pass, time K more steps with the "
                  "lanes carried across steps (a serving loop: step i + 1's "
                  "prefill overlaps step i's decode) and report them as "
                  "value_serving; on by default for C3, whose value is the "
                  "single-request rate")
  ap.add_argument("--rehearsal", choices=["cpu"], default=None,
                  help="no GPU: the launch / sharding / input generation / "
                  "gather / max-over-ranks path of the bench over gloo with a "
                  "deterministic per-sample digest standing in for the model "
                  "(the CPU test of the self-spawned multi-rank path)")
  args = ap.parse_args(argv)
  for k, v in CONFIGS[args.config].items():
    if getattr(args, k) is None:
      setattr(args, k, v)
  if args.cpu_decode_steps is None:
    args.cpu_decode_steps = args.decode
  if args.serving_pass is None:
    args.serving_pass = args.config == "c3"
  return args


def launch_ranks(n: int, argv) -> int:
  """`python bench.py --gpus N` outside a launcher: starts N rank processes
  through torch.distributed.run on 127.0.0.1 (one per GPU: RANK / LOCAL_RANK
  / WORLD_SIZE in their environment) and returns their exit code.  Called
  before this process touches the GPU, and as a child process (never an
  exec), so the launcher's ranks are the only processes that open a
  device."""
  import socket
  import subprocess
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
         f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
         f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
  env = dict(os.environ)
  env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host
  return subprocess.call(cmd, env=env)


def prefill_rates(mb: int, tokens_per_sample: int, prefill_ms_max: float,
                  world: int) -> tuple[float, float]:
  """(aggregate, per-rank) prefill tokens/s: every rank prefills `mb` samples
  of `tokens_per_sample` tokens in the timed micro-batch, and the slowest
  rank's prefill time bounds the job (global prefill tokens / max-over-ranks
  prefill time, SURVEY §8d: the >= 6x target is on the aggregate)."""
  per_rank = mb * tokens_per_sample / (prefill_ms_max * 1e-3)
  return per_rank * world, per_rank


def build_model(dev, image_size, text_only):
  torch.manual_seed(0)
  cfg = common.GriffinConfig.from_preset(common.Preset.RECURRENT_GEMMA_2B_V1)
  vis = None if text_only else common.VisionConfig(image_size=image_size)
  with torch.no_grad():
    model = cadence.Griffin(cfg, device=dev, dtype=torch.bfloat16, vision=vis)
  model.eval()
  return cfg, vis, model


def make_inputs(global_batch, lo, hi, image_size, prompt, vocab, text_only):
  """Rank-local slice [lo, hi) of the global synthetic batch: prompt tokens
  from one seeded stream over the whole batch (so every rank agrees), the
  images generated per rank from a seed of its first sample."""
  g = torch.Generator().manual_seed(4321)
  tok = torch.randint(3, vocab, (global_batch, prompt), generator=g,
                      dtype=torch.int32)
  tok[:, 0] = BenchVocab().bos_id()
  images = None
  if not text_only:
    # one seeded stream per global sample index: any sharding of the batch
    # over any number of ranks sees the same images
    images = torch.empty(hi - lo, 3, image_size, image_size)
    for i in range(lo, hi):
      gi = torch.Generator().manual_seed(1234 + i)
      images[i - lo] = torch.rand(3, image_size, image_size, generator=gi)
  return tok[lo:hi].contiguous(), images


def shard_plan(global_batch, micro_batch, rank, world, lanes=1):
  """(lo, hi, micro-batch slices) of the samples `rank` runs: a contiguous
  block of the global batch, cut into micro-batches of `micro_batch`.  With
  `lanes` > 1 (the two-lane generate_many pipeline) a rank whose share is ONE
  micro-batch runs it as `lanes` equal parts instead, so one part's prefill
  overlaps another's decode (lab option for the N = 8 point of the
  256-sample strong-scaling curve, 32 samples per rank: 2 x 16 measured
  slower than 1 x 32, profiles/r04c_n8_load_*)."""
  lo, hi = D.shard_range(global_batch, rank, world)
  if (hi - lo) % micro_batch:
    raise ValueError(f"{hi - lo} samples per rank is not a multiple of the "
                     f"micro-batch {micro_batch}")
  n = (hi - lo) // micro_batch
  if n == 1 and lanes > 1 and micro_batch % lanes == 0:
    micro_batch //= lanes
    n = lanes
  return lo, hi, [slice(j * micro_batch, (j + 1) * micro_batch) for j in range(n)]


def cpu_model_name():
  try:
    with open("/proc/cpuinfo") as f:
      for line in f:
        if line.startswith("model name"):
          return line.split(":", 1)[1].strip()
  except OSError:
    pass
  return None


def pmc_traffic(key, config="bench"):
  """Per-launch HBM bytes of `key` from the newest committed PMC summary of
  the same workload (profiles/*_pmc_traffic.json, written by
  tools/pmc_traffic.sh from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
  this bench; summaries without a "config" field are the default one), or
  None."""
  import glob
  files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
  for f in reversed(files):
    try:
      with open(f) as fh:
        d = json.load(fh)
    except (OSError, ValueError):
      continue
    if d.get("config", "bench") != config:
      continue
    k = d.get("kernels", {}).get(key)
    if k and k.get("hbm_bytes_per_launch"):
      return float(k["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
  return None


def roofline_entry(summary, key, bound, config="bench"):
  s = summary.get(key)
  if not s or s["avg_ms"] <= 0:
    return None
  if bound == "hbm":
    achieved = s["avg_work"] / (s["avg_ms"] * 1e-3) / 1e9
    peak, unit = HBM_PEAK_GBS, "GB/s"
  else:
    achieved = s["avg_work"] / (s["avg_ms"] * 1e-3) / 1e12
    peak, unit = MFMA_BF16_PEAK_TFS, "TFLOP/s"
  tr = pmc_traffic(key, config)
  return {"kernel": key, "bound": bound, "achieved": round(achieved, 2),
          "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
          "traffic": round(tr[0]) if tr else None,
          "traffic_source": (f"{tr[1]}: bytes/launch, 2*FETCH_SIZE + WRITE_SIZE "
                             "(fabric-side, Infinity-Cache hits included)") if tr else None,
          "avg_us": round(s["avg_ms"] * 1e3, 2),
          "launches_timed": s["launches"],
          "work_per_launch": s["avg_work"]}


def decode_hbm_bytes(model, cfg, batch, ctx_lens, window):
  """Algorithmic HBM bytes of ONE decode token-step for the whole batch:
  every Griffin weight once (blocks + final norm + the tied embedding the
  logits GEMM streams; the packed decode copies hold the same bytes), the
  KV-cache reads of the local-attention blocks at the replayed context
  lengths `ctx_lens` (mean), and the fp32 RG-LRU state read + write."""
  wbytes = sum(p.numel() * p.element_size() for n, p in model.named_parameters()
               if not n.startswith(("vis_encoder", "projector")))
  kinds = [k.name for k in cfg.block_types[:cfg.num_layers]]
  n_attn = kinds.count("ATTENTION")
  n_rec = len(kinds) - n_attn
  hd = cfg.width // cfg.num_heads
  ctx = sum(min(c, window) for c in ctx_lens) / len(ctx_lens)
  kv = n_attn * batch * ctx * 2 * hd * 2            # K and V, 1 kv head, bf16
  state = n_rec * batch * cfg.lru_width * 4 * 2      # h read + write, fp32
  return wbytes + kv + state


def vit_attention_isolated(vis, batch, dev, reps=20):
  """ViT attention alone (bench shapes, random qkv), HIP events around
  `reps` back-to-back launches on the current stream: in the step the two
  towers share the GPU, which stretches per-launch event windows."""
  out = {}
  for c in (vis.dino, vis.siglip):
    n = vis.n_visual_tokens + c.num_prefix_tokens
    qkv = torch.randn(batch * n, 3 * c.width, device=dev).to(torch.bfloat16)
    ops.ops.vit_attention(qkv, batch, n, c.num_heads, c.head_dim)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
      ops.ops.vit_attention(qkv, batch, n, c.num_heads, c.head_dim)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    flops = 4.0 * batch * c.num_heads * n * n * c.head_dim
    tf = flops / (us * 1e-6) / 1e12
    # q|k|v read once + output written once: at bs=32 these bytes take
    # longer at HBM peak than the FLOPs at MFMA peak, which caps the MFMA
    # fraction any kernel of this shape can reach (mfma_frac_ceiling)
    nbytes = batch * n * (3 * c.width + c.width) * 2
    t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
    t_mfma = flops / (MFMA_BF16_PEAK_TFS * 1e12)
    out[c.name] = {"kernel": ops.vit_attention_kernel_name(n, c.head_dim), "bound": "mfma",
                   "achieved": round(tf, 2), "peak": MFMA_BF16_PEAK_TFS,
                   "unit": "TFLOP/s", "frac": round(tf / MFMA_BF16_PEAK_TFS, 4),
                   "avg_us": round(us, 2), "work_per_launch": flops,
                   "shape": f"B={batch} N={n} H={c.num_heads} hd={c.head_dim}",
                   "hbm_bytes": nbytes,
                   "hbm_achieved": round(nbytes / (us * 1e-6) / 1e9, 1),
                   "hbm_frac": round(nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                   "mfma_frac_ceiling": round(t_mfma / max(t_mfma, t_hbm), 4),
                   "timing": f"isolated, {reps} launches after the timed region"}
  return out


def scan_isolated(batch, length, width, dev, reps=20):
  """rnn_scan alone at the workload's recurrent shape (x, a, the y gate in;
  y out; fp32 state out), HIP events around `reps` launches after the timed
  region: the prefill path now runs the scan inside the fused gates + scan
  kernel (rglru_scan_fused_kernel, VALU-bound by the gate chain), so the
  scan kernel's own HBM fraction -- the north star's RG-LRU scan bar -- is
  measured here; the same kernel runs where the fused plan does not apply
  (C3, small batches) and behind the public rnn_scan API."""
  g = torch.Generator(device=dev).manual_seed(5)
  m = batch * length
  x = torch.randn(m, width, device=dev, generator=g).to(torch.bfloat16)
  a = torch.rand(m, width, device=dev, generator=g).to(torch.bfloat16)
  gate = torch.randn(m, width, device=dev, generator=g).to(torch.bfloat16)
  run = lambda: ops.ops.rnn_scan(x, a, None, None, gate, batch, length)
  run()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  s.record()
  for _ in range(reps):
    run()
  e.record()
  torch.cuda.synchronize()
  us = s.elapsed_time(e) / reps * 1e3
  nbytes = m * width * 8 + batch * width * 4
  from cadence import _lib
  chunked = _lib.load().cadence_rnn_scan_workspace_bytes(batch, length, width) > 0
  gbs = nbytes / (us * 1e-6) / 1e9
  return {"kernel": "rnn_scan_chunk_kernel" if chunked else "rnn_scan_kernel",
          "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
          "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
          "avg_us": round(us, 2), "work_per_launch": nbytes,
          "shape": f"B={batch} L={length} E={width}",
          "timing": f"isolated, {reps} launches after the timed region; 8 B per "
                    "element (x, a, y gate in, y out, bf16) + fp32 state out"}


def image_preprocess_isolated(batch, size, dev, reps=20, h=480, w=640):
  """img_path preprocessing (Resize((S,S), BICUBIC) + ToTensor, Pillow-exact)
  on `batch` synthetic h x w RGB uint8 images already resident in HBM, HIP
  events around `reps` launches after the timed region; beside it Pillow's
  host resize of the same images (the reference's transform, one core,
  image by image as VisionEncoder.forward runs it)."""
  import numpy as np
  from PIL import Image
  from cadence import image_io
  rng = np.random.default_rng(99)
  arrs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for _ in range(batch)]
  meta = torch.tensor([[i * h * w * 3, h, w, i * h * size * 3] for i in range(batch)],
                      dtype=torch.int64, device=dev)
  packed = torch.from_numpy(np.concatenate([a.reshape(-1) for a in arrs])).to(dev)
  ks = max(ops.resize_taps(h, size), ops.resize_taps(w, size))
  run = lambda: torch.ops.cadence.resize_bicubic(packed, meta, size, ks, h, w,
                                                 batch * h * size * 3)
  run()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  s.record()
  for _ in range(reps):
    run()
  e.record()
  torch.cuda.synchronize()
  us = s.elapsed_time(e) / reps * 1e3
  nbytes = batch * (h * w * 3 + 3 * size * size * 4)     # u8 in + fp32 out
  gbs = nbytes / (us * 1e-6) / 1e9
  t0 = time.perf_counter()
  for a in arrs[:8]:
    Image.fromarray(a).resize((size, size), Image.BICUBIC)
  host_s = (time.perf_counter() - t0) / 8
  return {"kernel": "resize_coeff + resize_rows + resize_cols", "bound": "hbm",
          "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
          "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_us": round(us, 2),
          "work_per_launch": nbytes, "images_per_s": round(batch / (us * 1e-6), 1),
          "shape": f"B={batch} {h}x{w} -> {size}x{size}",
          "cpu_pillow_images_per_s": round(1.0 / host_s, 1),
          "timing": f"isolated, {reps} launches after the timed region; "
                    "algorithmic bytes = u8 input + fp32 output"}


def cpu_baseline(model, cfg, vis, tokens, images, decode_steps, budget_s=30.0):
  """The oracle (reference op sequence, B = 1 like the reference) on host
  cores, on a bounded sample: samples 0, 1, ... of the workload one at a time
  (full image + prompt prefill, `decode_steps` greedy decode steps each),
  up to min(B, 4) samples, starting another only while the
  projected total stays within `budget_s` of CPU time (the harness's 10-30 s
  bound for the sample; the first sample always runs)."""
  from oracle import griffin_ref as R
  # the host cores this process may use, capped by the box's CPU share
  # (OMP_NUM_THREADS = 16 per GPU there: sched_getaffinity sees the machine)
  cores = min(len(os.sched_getaffinity(0)), int(os.environ.get(
      "OMP_NUM_THREADS", "16") or 16))
  torch.set_num_threads(cores)
  p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
  n_vis = 0 if vis is None else vis.n_visual_tokens
  ntok = n_vis + tokens.shape[1] + decode_steps
  dt, n = 0.0, 0
  while n < min(tokens.shape[0], 4) and (n == 0 or dt * (n + 1) / n <= budget_s):
    tok = tokens[n:n + 1].cpu().long()
    px = None if images is None else images[n:n + 1].cpu()
    t0 = time.perf_counter()
    R.greedy_sample(p, cfg, tok, decode_steps, pixels=px, vcfg=vis)
    dt += time.perf_counter() - t0
    n += 1
  return {"value": round(n * ntok / dt, 2), "unit": "tokens/s", "cores": cores,
          "kind": "port", "cpu_model": cpu_model_name(),
          "sample": (f"{n} sample(s) run one at a time (B=1, the reference "
                     f"cannot batch; up to min(B, 4) within a {budget_s:.0f} s "
                     f"budget, the harness's 10-30 s bound): {n_vis} image + "
                     f"{tokens.shape[1]} prompt tokens prefill + {decode_steps} "
                     f"decode steps each, {dt:.1f} s"),
          "samples": n, "seconds": round(dt, 2)}


def rehearsal_rows(tok, img, decode, vocab):
  """Stand-in for one micro-batch's generated tokens in the CPU rehearsal: a
  deterministic function of each sample's prompt and image only, so the
  gathered rows of any sharding equal a one-rank run's."""
  base = tok.long().sum(1)
  if img is not None:
    base = base + (img * 255).round().long().flatten(1).sum(1)
  steps = torch.arange(decode, dtype=torch.int64)
  return ((base[:, None] * 31 + steps[None] * 7919) % vocab).to(torch.int32)


def rehearse(args):
  """--rehearsal cpu: the bench's multi-rank plumbing without a GPU (gloo):
  launch, shard_plan, make_inputs, the per-step gather, max-over-ranks timing
  and rank 0's JSON line (n_gpus, checksum, aggregate prefill rate)."""
  rank, world, _ = D.init_from_env(backend="gloo")
  if world != args.gpus:
    raise RuntimeError(f"--gpus {args.gpus} but the process group has {world} ranks")
  vocab = 256000
  gb = args.global_batch or args.batch * world
  lo, hi, micro = shard_plan(gb, args.batch, rank, world)
  tok, img = make_inputs(gb, lo, hi, args.image_size, args.prompt, vocab,
                         args.text_only)
  n_vis = 0 if args.text_only else (args.image_size // 14) ** 2
  D.barrier()
  t0 = time.perf_counter()
  tp = 0.0
  for _ in range(args.steps):
    outs = []
    for sl in micro:
      t1 = time.perf_counter()
      outs.append(rehearsal_rows(tok[sl], None if img is None else img[sl],
                                 args.decode, vocab))
      tp = time.perf_counter() - t1
    out = D.gather_rows(torch.cat(outs))
  D.barrier()
  own = time.perf_counter() - t0
  elapsed = D.max_over_ranks(own)
  rank_ms = D.all_over_ranks(own / args.steps * 1e3)
  rank_prefill_ms = D.all_over_ranks(tp * 1e3)
  mb = micro[0].stop - micro[0].start
  agg, per = prefill_rates(mb, n_vis + args.prompt, D.max_over_ranks(tp) * 1e3 + 1e-6,
                           world)
  tok_per_step = gb * (n_vis + args.prompt + args.decode)
  if rank == 0:
    print(json.dumps({
        "metric": "rehearsal (CPU, no model): " + METRIC, "n_gpus": world,
        "steps": args.steps, "value": round(gb * (n_vis + args.prompt + args.decode)
                                            * args.steps / elapsed, 2),
        "config": {"global_batch": gb, "micro_batch": mb,
                   "micro_batches_per_gpu": len(micro),
                   "parallelism": f"dp{world}"},
        "prefill_tokens_per_s": round(agg, 1),
        "prefill_tokens_per_s_per_rank": round(per, 1),
        "scaling_inputs": scaling_inputs(world, gb, tok_per_step,
                                         elapsed / args.steps * 1e3, rank_ms,
                                         rank_prefill_ms, agg),
        "definitions": DEFINITIONS,
        "generated_tokens_checksum": int(out.long().sum().item()),
        "gathered_rows": int(out.shape[0])}), flush=True)
  D.barrier()
  D.shutdown()


def fail_fast(exc: BaseException) -> None:
  """SURVEY §5 fail-fast: a rank that raises reports it, tears its process
  group down (bounded: a peer blocked in a collective cannot hold it) and
  exits non-zero, so the launcher stops the other ranks."""
  import threading
  import traceback
  rank = os.environ.get("RANK", "0")
  print(f"bench: rank {rank} failed: {exc!r}", file=sys.stderr)
  traceback.print_exc()
  sys.stderr.flush()
  sys.stdout.flush()
  t = threading.Thread(target=D.shutdown, daemon=True)
  t.start()
  t.join(timeout=10)
  os._exit(1)


def main(argv=None):
  args = parse(argv)
  in_launcher = "WORLD_SIZE" in os.environ
  if args.gpus > 1 and not in_launcher:
    # before any GPU call: this process only launches the ranks
    sys.exit(launch_ranks(args.gpus, sys.argv[1:] if argv is None else argv))
  try:
    if args.rehearsal:
      rehearse(args)
    else:
      run(args)
  except Exception as e:  # noqa: BLE001 -- every failure ends the job
    fail_fast(e)


def run(args):
  rank, world, local = D.init_from_env()
  if world != args.gpus:
    raise RuntimeError(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch with "
                       f"torch.distributed.run --nproc-per-node {args.gpus}, or "
                       f"run `python bench.py --gpus {args.gpus}` outside a "
                       "launcher and it starts the ranks itself")
  if torch.cuda.device_count() < world and os.environ.get(
      "CADENCE_DIST_BACKEND") != "gloo":
    raise RuntimeError(f"{world} ranks but {torch.cuda.device_count()} GPU(s) "
                       "visible (RCCL needs one GPU per rank)")
  dev = torch.device("cuda", D.local_device_index(local))
  torch.cuda.set_device(dev)
  if args.gemm_engine is not None:
    from cadence import _lib
    _lib.load().cadence_gemm_set_engine(args.gemm_engine)
  cfg, vis, model = build_model(dev, args.image_size, args.text_only)
  if os.environ.get("CADENCE_DUMP_MAPS"):
    # crash forensics (tools/pmc_crash_repro.sh): the process's library map,
    # once every library is loaded, so a native backtrace's addresses can be
    # resolved offline against the same image's libraries
    with open("/proc/self/maps") as fi, open(os.environ["CADENCE_DUMP_MAPS"], "w") as fo:
      fo.write(fi.read())
  n_vis = 0 if vis is None else vis.n_visual_tokens
  strong = bool(args.global_batch)
  gb = args.global_batch if strong else args.batch * world
  pipelined_plan = bool(args.decode and not args.no_pipeline and args.split_single)
  lo, hi, micro = shard_plan(gb, args.batch, rank, world,
                             lanes=2 if pipelined_plan else 1)
  n_micro = len(micro)
  # the lanes carried across steps where a step is one micro-batch (C2, a
  # rank's share at N = 8: 107 -> 95 ms per step); with several
  # micro-batches per step the lanes already overlap inside it (N = 1:
  # neutral, 747 vs 746 ms) and a continuous headline pass skews the
  # sequential pass's decode timing (profiles/r04zm_*).  C3 is a latency
  # config: its value is one request at a time, the two-requests-in-flight
  # rate goes to value_serving (--serving-pass)
  can_continue = bool(args.decode and not args.no_pipeline and n_micro == 1)
  continuous = can_continue and not args.no_continuous and not args.serving_pass
  mb = micro[0].stop - micro[0].start          # samples per micro-batch
  tok_cpu, img_cpu = make_inputs(gb, lo, hi, args.image_size, args.prompt,
                                 cfg.vocab_size, args.text_only)
  tokens = tok_cpu.to(dev)
  images = None if img_cpu is None else img_cpu.to(dev)
  lengths = torch.full((mb,), args.prompt, dtype=torch.int32)
  sampler = cadence.Sampler(model, BenchVocab(), use_graph=True)
  positions = torch.arange(args.prompt, dtype=torch.int32, device=dev)[None].repeat(
      mb, 1)

  gather_stream = torch.cuda.Stream()
  # under a process group the continuous loop is issued from its own
  # stream, not the null stream: an event on the legacy null stream waits
  # for every blocking stream (RCCL's among them), which chains step i + 1's
  # lanes to step i's all-gather (a rank's N = 8 load under an RCCL group of
  # one: 111 ms per step from the null stream, 94 from its own stream,
  # 104 without the continuous lanes; profiles/r04za_*).  Without a group
  # the null stream measured faster (96-98 vs 109 ms).  The inputs are made
  # before the timed loop.
  issue_stream = (torch.cuda.Stream() if torch.distributed.is_available() and
                  torch.distributed.is_initialized() else torch.cuda.current_stream())
  # the model's packing kernels and the input copies ran on the current
  # stream: the issue stream starts after them whatever those copies were
  issue_stream.wait_stream(torch.cuda.current_stream())
  plan = os.environ.get("CADENCE_QUEUE_PLAN")
  if plan:
    # lab: bind the lanes (L0, L1), their SigLIP side streams (S0, S1), the
    # gather stream (G) and spare pool streams (d) to hardware queues in the
    # given first-use order, e.g. "L0,L1,S0,d,S1,G" (profiles/r05k_hw_queue_lab.log)
    lanes = [torch.cuda.Stream(), torch.cuda.Stream()]
    sides = [torch.cuda.Stream(), torch.cuda.Stream()]
    roles = {"L0": lanes[0], "L1": lanes[1], "S0": sides[0], "S1": sides[1],
             "G": gather_stream}
    for tok in plan.split(","):
      st = roles.get(tok) or torch.cuda.Stream()
      st.wait_stream(torch.cuda.current_stream())
      with torch.cuda.stream(st):
        torch.zeros(1, device=dev).add_(1)
    sampler.__dict__["_lanes"] = {sampler.device: lanes}
    if getattr(model, "vis_encoder", None) is not None:
      model.vis_encoder.__dict__["_sides"] = {
          (dev, lanes[0].cuda_stream): sides[0], (dev, lanes[1].cuda_stream): sides[1]}
    torch.cuda.synchronize()

  def step(events=None, pipeline=True, done_event=None, lanes_across=None):
    if lanes_across is None:
      lanes_across = continuous
    if pipeline and can_continue and lanes_across:
      # a serving loop: micro-batches take the two lanes in turn across
      # steps (Sampler.generate_many continuous), so micro-batch j + 1's
      # prefill overlaps micro-batch j's decode also across a step boundary
      # (at N = 8 a rank's one micro-batch per step overlaps the next
      # step's); the step's rows are gathered on their own stream once both
      # lanes have produced them.  `events` time the last micro-batch
      with torch.cuda.stream(issue_stream):
        sts = sampler.generate_many(
            [(tokens[sl], lengths, None if images is None else images[sl])
             for sl in micro], args.decode, events=events, continuous=True)
      sampler.hand_over(sts, gather_stream)
      with torch.cuda.stream(gather_stream):
        out = D.gather_rows(torch.cat([st.tokens_buffer for st in sts]))
        if done_event is not None:
          done_event.record()
      return out
    # (one micro-batch has nothing to overlap: plain Sampler.generate)
    if args.decode and pipeline and not args.no_pipeline and n_micro > 1:
      # micro-batch j + 1's prefill overlaps micro-batch j's decode
      # (Sampler.generate_many); `events` time the last micro-batch
      sts = sampler.generate_many(
          [(tokens[sl], lengths, None if images is None else images[sl])
           for sl in micro], args.decode, events=events)
      return D.gather_rows(torch.cat([st.tokens_buffer for st in sts]))
    outs = []
    for j, sl in enumerate(micro):
      # the last micro-batch: by then the host has run ahead of the GPU, so
      # its prefill events time the GPU, not the launch loop (the first
      # micro-batch of a step starts on an empty queue)
      ev = events if j == n_micro - 1 else None
      if args.decode == 0 and ev is not None:    # prefill only (C4)
        ev["prefill_start"] = torch.cuda.Event(enable_timing=True)
        ev["prefill_end"] = torch.cuda.Event(enable_timing=True)
        ev["prefill_start"].record()
      img = None if images is None else images[sl]
      if args.decode == 0:
        # prefill only (C4): the forward over [image | prompt] that builds
        # the caches (Sampler.generate with 0 steps would skip it, as the
        # reference's return_logits=False / return_cache=False forward does)
        _, cache = model(tokens[sl], positions, images=img,
                         return_logits=False, return_cache=True,
                         image_splice=img is not None)
        if ev is not None:
          ev["prefill_end"].record()
        outs.append(cache["blocks.0"][0][:, :1].float().to(torch.int32))
        continue
      st = sampler.generate(tokens[sl], lengths, args.decode, images=img,
                            events=ev)
      outs.append(st.tokens_buffer)
    return D.gather_rows(torch.cat(outs))

  host_enqueue = {}

  def timed_pass(kernel_timing: bool, lanes_across=None):
    """K steps between barrier + synchronize; with kernel_timing a seeded
    1/4 of the prefill GEMM / attention / scan launches carry HIP events on
    their stream (ops.TIMER).  Returns (seconds, step events, per-step
    prefill/decode events, last output)."""
    # ~400 timed launches per micro-batch; a seeded 1/4 of them carry events
    ops.TIMER.reset(pool=250 * args.steps * n_micro if kernel_timing else 0,
                    sample=4)
    ops.TIMER.enabled = kernel_timing
    evs = []
    sev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sev[0].record()
    o = None
    for i in range(args.steps):
      ev = {}
      # the kernel-timing pass runs the micro-batches one after another: with
      # two lanes in flight an event pair would also time the queueing behind
      # the other lane's kernels, not the launch itself
      across = continuous if lanes_across is None else lanes_across
      o = step(ev, pipeline=not kernel_timing, done_event=sev[i + 1],
               lanes_across=across)
      if not (across and can_continue and not kernel_timing):
        sev[i + 1].record()
      evs.append(ev)
    # host time to enqueue the K steps (no sync inside a step): under the
    # device time means the host runs ahead and the GPU does not wait on it
    host_enqueue["s"] = time.perf_counter() - t0
    torch.cuda.synchronize()
    D.barrier()
    t1 = time.perf_counter()
    ops.TIMER.enabled = False
    return t1 - t0, sev, evs, o

  with torch.no_grad():
    serving = None
    if args.serving_pass and can_continue:
      # C3's serving loop over K steps: the lanes carried across steps, two
      # requests in flight (one prefills while the other decodes); each lane
      # captures its decode graph on its first micro-batch, which must not
      # fall in the timed steps.  It runs BEFORE the single-request passes:
      # HIP binds a stream to one of the GPU_MAX_HW_QUEUES = 4 hardware
      # queues at its first use (the least used, ties to the last), and after
      # the single-request pass had bound its own streams (the SigLIP side
      # stream of the caller's stream, a decode-graph capture stream) the
      # serving loop measured 58 ms per step instead of 44 -- by the binding
      # rule tools/hw_queue_map.py measures, its two lanes then share one
      # queue (profiles/r05k_hw_queue_lab.log)
      for _ in range(max(args.warmup, 2)):
        step(lanes_across=True)
      torch.cuda.synchronize()
      sdt, _, _, _ = timed_pass(False, lanes_across=True)
      serving = D.max_over_ranks(sdt)
    # the continuous lanes take one micro-batch per step in turn: each lane
    # captures its decode graph on its first micro-batch, so the untimed
    # warmup covers at least one step per lane
    for _ in range(max(args.warmup, 2) if continuous else args.warmup):
      out = step()
    torch.cuda.synchronize()
    # the headline pass carries no per-kernel events (they cost the stream
    # ~3 % of the step); a second pass of the same K steps times the kernels
    dt, step_ev, ev_list, out = timed_pass(False)
    host_ms = host_enqueue["s"] * 1e3 / args.steps
    ksum = {}
    pipelined = bool(args.decode and not args.no_pipeline and (n_micro > 1 or continuous))
    if not args.no_kernel_timing:
      _, _, ev_seq, _ = timed_pass(True)
      ksum = ops.TIMER.summary()
      # with two lanes in flight the headline pass's prefill / decode event
      # pairs would time queueing behind the other lane: take them from the
      # sequential pass then (otherwise from the headline pass, which carries
      # no per-kernel events: a B = 1 prefill is launch-bound, and the
      # events would inflate it)
      if pipelined:
        ev_list = ev_seq
  elapsed = D.max_over_ranks(dt)
  # with the lanes carried across steps (continuous) consecutive steps
  # finish alternately early and late: the median is taken over
  # non-overlapping two-step windows (per step)
  win = 2 if (continuous and args.steps >= 2) else 1
  per_step = sorted(step_ev[i].elapsed_time(step_ev[i + win]) / win
                    for i in range(0, args.steps + 1 - win, win))
  mid = len(per_step) // 2
  median_ms = D.max_over_ranks(per_step[mid] if len(per_step) % 2 else
                               0.5 * (per_step[mid - 1] + per_step[mid]))
  prefill_ms = []
  decode_ms = []
  for ev in ev_list:
    prefill_ms.append(ev["prefill_start"].elapsed_time(ev["prefill_end"]))
    if "decode_start" in ev:
      decode_ms.append(ev["decode_start"].elapsed_time(ev["decode_end"])
                       / ev["decode_steps"])
  vit_iso = (vit_attention_isolated(vis, args.batch, dev)
             if vis is not None and rank == 0 and not args.no_kernel_timing else None)
  img_iso = (image_preprocess_isolated(args.batch, args.image_size, dev)
             if vis is not None and rank == 0 and not args.no_kernel_timing else None)
  scan_iso = None
  if (rank == 0 and not args.no_kernel_timing and not any(
      k in ksum for k in ("rnn_scan_kernel", "rnn_scan_chunk_kernel"))):
    scan_iso = scan_isolated(mb, n_vis + args.prompt - (1 if args.decode else 0),
                             cfg.lru_width, dev)

  tok_per_step = gb * (n_vis + args.prompt + args.decode)
  value = tok_per_step * args.steps / elapsed
  ms_step = elapsed / args.steps * 1e3
  pre_ms = sum(prefill_ms) / max(len(prefill_ms), 1)
  pre_ms = D.max_over_ranks(pre_ms)
  prefill_tps, prefill_tps_rank = prefill_rates(
      mb, n_vis + args.prompt - (1 if args.decode else 0), pre_ms, world)

  # every rank's own end-to-end time per step (the driver's speed-up input
  # on `value`) and its prefill time, gathered before rank 0 prints
  rank_ms = D.all_over_ranks(dt / args.steps * 1e3)
  rank_prefill_ms = D.all_over_ranks(sum(prefill_ms) / max(len(prefill_ms), 1))
  result = None
  fused_scan = next((roofline_entry(ksum, k, "hbm", args.config) for k in sorted(ksum)
                     if k.startswith("rglru_scan_fused_kernel")), None)
  if rank == 0:
    # dominant kernel: the single-stream GEMM key with the most time in the
    # step (ViT-tower launches share the GPU between two streams: their keys
    # carry a " [vit, 2 streams]" suffix and are reported, not ranked)
    gemm_keys = [k for k in ksum if k.startswith(("gemm_big_kernel", "gemm_w4_kernel"))
                 and "[" not in k]
    dom = max(gemm_keys, key=lambda k: ksum[k]["total_ms"]) if gemm_keys else None
    # the prefill scan: the sequential kernel (B * E / 2 lanes fill the chip)
    # or the T-chunked one (small batches)
    scan_keys = [k for k in ("rnn_scan_kernel", "rnn_scan_chunk_kernel") if k in ksum]
    scan_key = max(scan_keys, key=lambda k: ksum[k]["total_ms"]) if scan_keys else None
    dec = None
    if decode_ms:
      # replayed steps: the last `decode_steps` of the prompt-token step +
      # decode steps; step i attends to n_vis + prompt + i keys
      dsteps = ev_list[0]["decode_steps"]
      ctx = [n_vis + args.prompt + i for i in range(args.decode - dsteps, args.decode)]
      nbytes = decode_hbm_bytes(model, cfg, mb, ctx,
                                cfg.attention_window_size)
      us = sum(decode_ms) / len(decode_ms) * 1e3
      gbs = nbytes / (us * 1e-6) / 1e9
      dec = {"kernel": "decode token-step (hipGraph, all kernels)",
             "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
             "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
             "avg_us": round(us, 1), "work_per_launch": nbytes}
    what = ("text-only" if args.text_only else f"{args.image_size}px")
    metric = METRIC if args.config == "bench" else (
        f"{'text-only' if args.text_only else 'multimodal'} prefill"
        f"{'+decode' if args.decode else ''} tokens/sec, Cadence-2B {what} "
        f"bs={args.batch} (SURVEY §8d {args.config.upper()})")
    result = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "ms_per_step_median": round(median_ms, 3),
        "host_enqueue_ms_per_step": round(host_ms, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": ("synthetic: torch.rand images (seeded per sample), random "
                 "prompt tokens (seed 4321), random-init weights (seed 0)"),
        "config": {
            "workload": ("Cadence-2B (RecurrentGemma-2B + DINOv2-L/14-reg4 + "
                         "SigLIP-so400m/14 + MLP projector) " + what +
                         f", global batch {gb} = {world} GPU(s) x {n_micro} "
                         f"micro-batch(es) of {mb}, prompt "
                         f"{args.prompt}, greedy decode {args.decode}"),
            "config": args.config,
            "global_batch": gb, "micro_batch": mb,
            "micro_batches_per_gpu": n_micro,
            "image_size": None if args.text_only else args.image_size,
            "n_visual_tokens": n_vis,
            "prompt_len": args.prompt, "decode_steps": args.decode,
            "seq_len": n_vis + args.prompt + args.decode,
            "parallelism": f"dp{world}",
            "micro_batch_pipeline": bool(args.decode and not args.no_pipeline
                                         and (n_micro > 1 or continuous)),
            "requests_in_flight": 2 if continuous else (1 if n_micro == 1 else n_micro),
            "pipeline_across_steps": continuous,
        },
        "prefill_ms": round(pre_ms, 3),
        "prefill_timing": (("last micro-batch's prefill in the kernel-timing pass "
                            "(micro-batches run one after another)"
                            if not args.no_kernel_timing else
                            "last micro-batch's prefill, overlapping the previous "
                            "micro-batch's decode (Sampler.generate_many)")
                           if args.decode and not args.no_pipeline and
                           (n_micro > 1 or continuous)
                           else "last micro-batch's prefill (headline pass)"),
        "prefill_tokens_per_s": round(prefill_tps, 1),
        "prefill_tokens_per_s_per_rank": round(prefill_tps_rank, 1),
        "prefill_tokens_per_s_definition": (
            "aggregate over ranks: world x micro-batch x prefill tokens per "
            "sample / max-over-ranks prefill time of the timed micro-batch"),
        "scaling_inputs": scaling_inputs(world, gb, tok_per_step, ms_step, rank_ms,
                                         rank_prefill_ms, prefill_tps),
        "definitions": DEFINITIONS,
        "roofline": roofline_entry(ksum, dom, "mfma", args.config) if dom else None,
        # the RG-LRU scan the workload runs: the scan kernel where the
        # headline launches it, else the fused gates + scan kernel (HBM-priced
        # on x and the y gate in, y out, weights and state; the gate chain's
        # VALU, not the bytes, bounds it)
        "roofline_scan": (roofline_entry(ksum, scan_key, "hbm", args.config)
                          if scan_key else fused_scan),
        "roofline_rglru_fused": fused_scan,
        # rnn_scan_kernel alone at the workload's shape (the small-batch /
        # rnn_scan API path), timed after the timed region: not a kernel the
        # headline runs when roofline_scan names the fused kernel
        "roofline_scan_isolated": scan_iso,
        "roofline_decode": dec,
        # prefill RG-LRU gates: HBM-priced (x in, a and normalised x out)
        "roofline_rglru_gates": next((roofline_entry(ksum, k, "hbm", args.config)
                                      for k in sorted(ksum)
                                      if k.startswith("rglru_gates_stream_kernel")), None),
        "roofline_vit_attention": vit_iso,
        "roofline_image_preprocess": img_iso,
        "roofline_by_kernel": {k: roofline_entry(ksum, k, "mfma", args.config)
                               for k in sorted(ksum)
                               if k.startswith(("gemm_big", "gemm_w4", "vit_attn",
                                                "vit_flash", "vit_stream", "flash_attn",
                                                "griffin_attn"))},
        # a seeded 1/sample of the launches is event-timed (TIMER.sample)
        "kernels": {k: {"launches_timed": v["launches"],
                        "avg_us": round(v["avg_ms"] * 1e3, 2),
                        "est_ms_per_step": round(v["total_ms"] * ops.TIMER.sample /
                                                 args.steps, 3)}
                    for k, v in sorted(ksum.items())},
        "kernel_timing": f"HIP events on a seeded 1/{ops.TIMER.sample} of the launches "
                         "of a second timed pass of the same K steps, micro-batches "
                         "run one after another (the value / ms_per_step pass "
                         "carries no per-kernel events: they cost the stream ~3 % "
                         "of the step; it runs two micro-batch lanes whose kernels "
                         "share the CUs, so an event pair there would time "
                         "queueing behind the other lane)",
        "generated_tokens_checksum": int(out.long().sum().item()),
    }
    if serving is not None:
      result["value_serving"] = round(tok_per_step * args.steps / serving, 2)
      result["ms_per_step_serving"] = round(serving / args.steps * 1e3, 3)
      result["value_serving_definition"] = (
          "the same K steps with the two lanes carried across steps (a serving "
          "loop: step i + 1's request prefills while step i's decodes; two "
          "requests in flight); value is one request at a time")
    if world == 1 and not args.no_cpu_baseline:
      result["cpu_baseline"] = cpu_baseline(model, cfg, vis, tok_cpu, img_cpu,
                                            args.cpu_decode_steps)
    else:
      result["cpu_baseline"] = None
    print(json.dumps(result), flush=True)
  D.barrier()
  D.shutdown()


if __name__ == "__main__":
  main()
