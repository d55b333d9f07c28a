#!/bin/bash
# Focused GPU check: one pytest selection, then a short rocprofv3 stats run
# of the default bench and the lines of the named kernels.
# usage: tools/focus_prof.sh TAG "PYTEST ARGS" "KERNEL REGEX"
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}; sel=${2:?pytest args}; rx=${3:?kernel regex}
tools/gpu_step.sh 300 ${tag}_focus.log python -u -m pytest $sel -q --tb=short --timeout 120 --timeout-method thread || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${tag}_prof.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 60 > gpurun_out/${tag}_kstats.txt
rm -rf gpurun_out/prof_$tag
grep '^{' gpurun_out/${tag}_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('value', d['value'], 'decode_us', d['roofline_decode']['avg_us'])"
grep -E "$rx" gpurun_out/${tag}_kstats.txt | cut -c1-140
