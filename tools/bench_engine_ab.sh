#!/bin/bash
# Bench prefill / per-kernel A/B of the GEMM engine plans: two bench runs
# (engine 0 = 8-wave only, 1 = shipped plan), the per-kernel averages side
# by side.  usage: tools/bench_engine_ab.sh TAG
tag=${1:?tag}
for e in 0 1 0 1; do
  tools/gpu_step.sh 300 ${tag}_e$e.log python -u bench.py --no-cpu-baseline --steps 3 --gemm-engine $e || exit 1
  mv gpurun_out/${tag}_e$e.log gpurun_out/${tag}_e${e}_$(date +%s%N).log
done
python3 - "$tag" <<'PY'
import glob, json, sys
tag = sys.argv[1]
for e in (0, 1):
  for f in sorted(glob.glob(f"gpurun_out/{tag}_e{e}_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][0])
    print(f"engine {e}: value {d['value']} prefill_ms {d['prefill_ms']} decode_us {d['roofline_decode']['avg_us']}")
    for k, v in sorted(d["kernels"].items()):
      if k.startswith("gemm"):
        print(f"   {k:60s} {v['avg_us']:8.1f} us  {v['est_ms_per_step']:8.2f} ms/step")
PY
