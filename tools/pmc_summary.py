"""Per-launch HBM traffic from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes
of tools/pmc_traffic.sh -> profiles/<tag>_pmc_traffic.json (read by bench.py).

HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 per launch (KiB
counters; gfx950 FETCH_SIZE counts half of a wide streaming read, per the
MI355X guide's HBM section).  Keys are the bench's kernel keys.

usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<tag>_pmc_traffic.json SOURCE
"""

import csv
import json
import re
import sys
from collections import defaultdict

# bench key -> (regex on the rocprof kernel name, algorithmic bytes per
# launch at the bench workload: 224 px, B = 32, L = 319, E = D = 2560)
KEYS = {
    "rnn_scan_kernel": (r"rnn_scan_kernel<", 8 * 32 * 319 * 2560 + 32 * 2560 * 4,
                        "x, a, gate in + y out (bf16) + fp32 h_last out"),
    "gemm_big_kernel<EpiGatedGelu, 1, 7>": (
        r"gemm_big_kernel<[^>]*EpiGatedGelu, 1, 7>",
        2 * (10208 * 2560 + 2 * 7680 * 2560 + 10208 * 7680),
        "A (M x K) + W (2F x K) + out (M x F), bf16"),
    "gemm_w4_kernel<EpiGatedGelu, 7>": (
        r"gemm_w4_kernel<[^>]*EpiGatedGelu, 7>",
        2 * (10208 * 2560 + 2 * 7680 * 2560 + 10208 * 7680),
        "A (M x K) + W (2F x K) + out (M x F), bf16"),
    "gemm_w4_kernel<EpiGatedGelu, 8>": (
        r"gemm_w4_kernel<[^>]*EpiGatedGelu, 8>",
        2 * (10208 * 2560 + 2 * 7680 * 2560 + 10208 * 7680),
        "A (M x K) + W (2F x K) + out (M x F), bf16"),
    "rglru_scan_fused_kernel<256>": (
        r"rglru_scan_fused_kernel<256", 6 * 10208 * 2560 + 10 * 512 * 256 * 2
        + 32 * 2560 * 4 + 10208 * 4,
        "x and the y gate in + y out (bf16) + packed gate weights + fp32 state out"),
    "rglru_gates_stream_kernel<256>": (
        r"rglru_gates_stream_kernel<256>", 3 * 10208 * 2560 * 2 + 10 * 512 * 256 * 2,
        "x in + a, normalised x out (bf16) + packed gate weights"),
    "gemm_gated_pipe_kernel<10, 2, 3, true> (decode)": (
        r"gemm_gated_pipe_kernel<10, 2, 3, true(, 2)?>", 79134720,
        "2F x K bf16 weights + activations + out"),
    "gemm_stream_kernel<32, 10, 2, EpiResidRows> (decode)": (
        r"gemm_stream_kernel<32, 10, 2, [^>]*EpiResidRows[^>]*>", 2560 * 7680 * 2,
        "N x K bf16 weights (down projection; activations, slabs, out extra)"),
}


def load(path):
  per = defaultdict(list)
  with open(path) as f:
    for r in csv.DictReader(f):
      per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
  return per


def main():
  d, out, source = sys.argv[1], sys.argv[2], sys.argv[3]
  fetch = load(f"{d}/pmc_FETCH_SIZE.csv")
  write = load(f"{d}/pmc_WRITE_SIZE.csv")
  res = {}
  for key, (rx, alg, note) in KEYS.items():
    names = [n for n in fetch if re.search(rx, n)]
    if not names:
      continue
    fv = [v for n in names for v in fetch[n]]
    wv = [v for n in names for v in write.get(n, [])]
    if not fv or not wv:
      continue
    fk, wk = sum(fv) / len(fv), sum(wv) / len(wv)
    res[key] = {"launches": len(fv), "fetch_size_kb": fk, "write_size_kb": wk,
                "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
                "algorithmic_bytes_per_launch": alg, "note": note}
  with open(out, "w") as f:
    json.dump({"source": source,
               "correction": "HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 "
                             "(gfx950 FETCH_SIZE counts half of a wide streaming read; "
                             "MI355X_MICROARCH.md HBM section). Infinity-Cache hits are "
                             "counted by these fabric-side counters.",
               "kernels": res}, f, indent=1)
  for k, v in res.items():
    print(f"{k:55s} {v['launches']:5d} {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB "
          f"(algorithmic {v['algorithmic_bytes_per_launch'] / 1e6:.1f} MB)")


if __name__ == "__main__":
  main()
