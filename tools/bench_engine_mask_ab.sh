#!/bin/bash
# in-pipeline engine A/B: value + gated GEMM per engine mask
for e in 3 2 3 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --gemm-engine $e > gpurun_out/r03p_e$e.log 2>&1 || exit 1
  python3 - "$e" <<'PY'
import json,sys
d=[json.loads(l) for l in open(f"gpurun_out/r03p_e{sys.argv[1]}.log") if l.startswith("{")][0]
g={k:v["avg_us"] for k,v in d["kernels"].items() if "Gated" in k or "rglru" in k}
print("engine", sys.argv[1], "value", d["value"], "prefill_ms", d["prefill_ms"], g, flush=True)
PY
done
