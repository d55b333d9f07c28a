#!/bin/bash
# Committed evidence for a round: full bench line (with cpu_baseline) and a
# rocprofv3 kernel-trace --stats run of the same bench command.
# usage: tools/profile_round.sh TAG   (outputs under gpurun_out/TAG/)
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.log > $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $out/kernel_stats.csv
python3 tools/prof_summary.py "$f" 40 > $out/kernel_stats.txt
grep '^{' $out/prof.log > $out/bench_under_rocprof.json
rm -rf $out/prof
cat $out/kernel_stats.txt | head -12
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['frac'], d['cpu_baseline'])"
