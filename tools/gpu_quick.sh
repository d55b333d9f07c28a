#!/bin/bash
# Quick GPU iteration: one test file, the whole GPU suite, a bench line and a
# short rocprofv3 kernel-stats run.  usage: tools/gpu_quick.sh TAG TESTFILE
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}; tf=${2:-}
S=tools/gpu_step.sh
if [ -n "$tf" ]; then
  $S 300 ${tag}_focus.log python -u -m pytest $tf -q --tb=short --timeout 120 --timeout-method thread || exit 1
fi
$S 600 ${tag}_pytest.log python -u -m pytest tests -m gpu -q --tb=short --timeout 300 --timeout-method thread || exit 1
$S 400 ${tag}_bench.log python -u bench.py --no-cpu-baseline || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${tag}_prof.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 40 > gpurun_out/${tag}_kstats.txt
cp "$f" gpurun_out/${tag}_kstats.csv
rm -rf gpurun_out/prof_$tag
python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][0]); print('value', d['value'], 'prefill_ms', d['prefill_ms'], 'decode_us', d['roofline_decode']['avg_us'], 'frac', d['roofline']['frac'])"
