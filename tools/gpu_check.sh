#!/bin/bash
# One GPU round: parity tests, bench, rocprofv3 kernel stats (CSV).
# usage: tools/gpu_check.sh [tag] [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-run}
mkdir -p gpurun_out
kexpr=${2:-}
if [ -n "$kexpr" ]; then kargs=(-k "$kexpr"); else kargs=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${kargs[@]}" > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -30 gpurun_out/bench_$tag.log; exit 1; }
grep '^{' gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms/step',d['ms_per_step'],'prefill_ms',d['prefill_ms']); [print(f'  {k:40s} {v}') for k,v in d['kernels'].items()]; [print(k, d.get(k)) for k in ('roofline','roofline_decode','roofline_vit_attention')]"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 30
