"""Launch gaps of the decode token-step (hipGraph replay, B = 32, 224 px).

  target:  python3 tools/decode_gaps.py [STEPS]    (under rocprofv3 --kernel-trace)
  summary: python3 tools/decode_gaps.py --summary KERNEL_TRACE.csv

The summary takes the dispatches after the prefill's last ViT / prefill GEMM
(the decode replays), splits them into token steps at each embedding
kernel, and reports per step: wall time (first start -> last end), the sum
of kernel durations, and the idle time between consecutive kernels -- the
part a chained (ticketed) decode layer could remove without touching any
kernel's own ramp.
"""

import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cadence-gemma_amd")]


def run(steps):
  import torch
  import bench
  import cadence
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  cfg, vis, model = bench.build_model(dev, 224, False)
  tok, img = bench.make_inputs(32, 0, 32, 224, 64, cfg.vocab_size, False)
  lengths = torch.full((32,), 64, dtype=torch.int32)
  sampler = cadence.Sampler(model, bench.BenchVocab(), use_graph=True)
  with torch.no_grad():
    for _ in range(2):   # the first call captures the decode graph
      st = sampler.generate(tok.to(dev), lengths, steps, images=img.to(dev))
  torch.cuda.synchronize()
  print("tokens checksum", int(st.tokens_buffer.long().sum().item()))


def summary(path):
  rows = list(csv.DictReader(open(path)))
  rows.sort(key=lambda r: int(r["Start_Timestamp"]))
  name = lambda r: r["Kernel_Name"]
  # the last call's decode: dispatches after its last prefill-only kernel
  last_prefill = max(i for i, r in enumerate(rows)
                     if "gemm_w4_kernel" in name(r) or "rglru_scan" in name(r))
  dec = rows[last_prefill + 1:]
  steps, cur = [], []
  for r in dec:
    if "embed_kernel" in name(r) and cur:
      steps.append(cur)
      cur = []
    cur.append(r)
  if cur:
    steps.append(cur)
  full = [s for s in steps if len(s) > 50]
  print(f"{len(full)} token steps, {sum(len(s) for s in full) / max(1, len(full)):.0f} "
        f"kernels per step")
  tot_wall = tot_busy = 0.0
  gaps = []
  for s in full[1:]:
    st = [int(r["Start_Timestamp"]) for r in s]
    en = [int(r["End_Timestamp"]) for r in s]
    wall = (max(en) - min(st)) / 1e3
    busy = sum(e - b for b, e in zip(st, en)) / 1e3
    g = [(st[i + 1] - en[i]) / 1e3 for i in range(len(s) - 1)]
    gaps += g
    tot_wall += wall
    tot_busy += busy
  n = max(1, len(full) - 1)
  gaps.sort()
  med = gaps[len(gaps) // 2] if gaps else 0.0
  print(f"per step: wall {tot_wall / n:.1f} us, kernel time {tot_busy / n:.1f} us, "
        f"idle between kernels {(tot_wall - tot_busy) / n:.1f} us "
        f"({100 * (tot_wall - tot_busy) / max(tot_wall, 1e-9):.1f} %); gap median {med:.2f} us, "
        f"p10 {gaps[len(gaps) // 10] if gaps else 0:.2f}, p90 {gaps[9 * len(gaps) // 10] if gaps else 0:.2f}")


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "--summary":
    summary(sys.argv[2])
  else:
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 12)
