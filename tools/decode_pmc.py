"""PMC traffic of today's decode kernels (verdict r05 item 7).

rocprofv3's PMC mode crashes on graph-replayed dispatches ("The
rocprofv3 PMC crash"), so this drives the bench's decode on the EAGER path:
the bench model and inputs (224 px, one micro-batch of 32, prompt 64), then
`Sampler(use_graph=False).generate` for STEPS greedy steps -- the same
kernels the hipGraph replays, launched one by one.

  target:  python3 tools/decode_pmc.py [STEPS]          (under rocprofv3 --pmc)
  summary: python3 tools/decode_pmc.py --summary DIR OUT.json

The summary reads DIR/pmc_FETCH_SIZE.csv and DIR/pmc_WRITE_SIZE.csv and
reports, per decode kernel, the mean per-launch HBM bytes = 2 x FETCH_SIZE +
WRITE_SIZE (KiB counters; gfx950 FETCH_SIZE counts half of a wide streaming
read, MI355X_MICROARCH.md "HBM") against the kernel's algorithmic bytes.
"""

import csv
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cadence-gemma_amd")]

B, D, F, E, H, HD, V = 32, 2560, 7680, 2560, 10, 256, 256000
# rocprof kernel-name regex -> (label, algorithmic bytes per launch at B = 32)
KERNELS = [
    (r"gemm_gated_pipe_kernel", "MLP gated up-projection (2F x D weights)", 2 * F * D * 2),
    (r"gemm_stream_kernel<[^>]*EpiResidRows", "MLP down projection, K splits combined in-kernel",
     D * F * 2),
    (r"gemm_stream_kernel<[^>]*EpiLinearConv", "recurrent y|x projection + Conv1D step",
     2 * E * D * 2),
    (r"gemm_stream_kernel<[^>]*EpiRopeQKV", "attention q|k|v projection + RoPE",
     (H + 2) * HD * D * 2),
    (r"gemm_resid_pipe_kernel", "output projections (residual epilogue)", D * D * 2),
    (r"gemm_stream_kernel<[^>]*EpiRglruGates|rglru_step", "RG-LRU gates GEMV + scan step",
     H * 2 * HD * HD * 2 + B * E * 4 * 2),
    (r"decode_attn_kernel", "decode attention (K/V ring at the replayed context)", None),
    (r"gemm_skinny_kernel", "logits (tied embedding)", V * D * 2),
]


def run(steps):
  import torch
  import bench
  import cadence
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  cfg, vis, model = bench.build_model(dev, 224, False)
  tok, img = bench.make_inputs(B, 0, B, 224, 64, cfg.vocab_size, False)
  lengths = torch.full((B,), 64, dtype=torch.int32)
  sampler = cadence.Sampler(model, bench.BenchVocab(), use_graph=False)
  with torch.no_grad():
    st = sampler.generate(tok.to(dev), lengths, steps, images=img.to(dev))
  torch.cuda.synchronize()
  print("tokens checksum", int(st.tokens_buffer.long().sum().item()))


def load(path):
  per = defaultdict(list)
  with open(path) as f:
    for r in csv.DictReader(f):
      per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
  return per


def summary(d, out):
  fetch, write = load(f"{d}/pmc_FETCH_SIZE.csv"), load(f"{d}/pmc_WRITE_SIZE.csv")
  res = {}
  for rx, label, alg in KERNELS:
    fk = [k for k in fetch if re.search(rx, k)]
    wk = [k for k in write if re.search(rx, k)]
    if not fk:
      continue
    fv = [v for k in fk for v in fetch[k]]
    wv = [v for k in wk for v in write[k]]
    f_kib = sum(fv) / len(fv)
    w_kib = sum(wv) / len(wv) if wv else 0.0
    hbm = (2 * f_kib + w_kib) * 1024
    res[label] = {"kernels": sorted(set(fk)), "launches": len(fv),
                  "fetch_kib": round(f_kib, 1), "write_kib": round(w_kib, 1),
                  "hbm_bytes": round(hbm), "algorithmic_bytes": alg,
                  "ratio": round(hbm / alg, 3) if alg else None}
  act = lambda k: 8 * B * k * 2   # packed activation rows fetched once per XCD (8 L2s)
  notes = {
      "MLP down projection, K splits combined in-kernel":
          f"extra over the weights ~ the [B, F] activations once per XCD ({act(F)} B) + "
          f"the 3 K splits' fp32 partials written and read back ({2 * 3 * B * D * 4} B) + "
          f"the residual rows in and out ({2 * B * D * 2} B)",
      "output projections (residual epilogue)":
          f"extra ~ the [B, D] activations once per XCD ({act(D)} B) + the residual "
          f"rows in and out ({2 * B * D * 2} B)",
      "recurrent y|x projection + Conv1D step":
          f"extra ~ the activations once per XCD ({act(D)} B), the Conv1D state read + "
          "written and the y / x outputs",
      "attention q|k|v projection + RoPE":
          f"extra ~ the activations once per XCD ({act(D)} B) and the q / k / v outputs",
      "RG-LRU gates GEMV + scan step":
          "algorithmic = block-diagonal gate weights + the fp32 RG-LRU state read and "
          "written; the rest is the [B, 2E] gate inputs and outputs",
      "decode attention (K/V ring at the replayed context)":
          "no algorithmic figure: the bytes follow the attended key range of each "
          "step (one K + V row per key, 1 KiB after the x2 correction, is the step-to-"
          "step increment seen in the per-launch counters)",
  }
  for k, v in res.items():
    if k in notes:
      v["note"] = notes[k]
  doc = {"source": "tools/decode_pmc.py: eager decode (Sampler use_graph=False), 224 px, "
                   "B = 32, separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes; "
                   "hbm = 2 x FETCH + WRITE (gfx950 correction)",
         "kernels": res}
  with open(out, "w") as f:
    json.dump(doc, f, indent=1)
  for k, v in res.items():
    print(f"{k:60s} {v['hbm_bytes'] / 1e6:9.2f} MB vs {(v['algorithmic_bytes'] or 0) / 1e6:9.2f}"
          f"  ratio {v['ratio']}  ({v['launches']} launches)")


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "--summary":
    summary(sys.argv[2], sys.argv[3])
  else:
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
