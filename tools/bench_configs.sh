#!/bin/bash
# The SURVEY §8d configurations besides the driver's default line:
# C2 (text-only, B=32, T=2048, 64 decode), C3 (224 px, B=1), C4 (336 px,
# B=32, prefill only), each with its roofline objects and cpu_baseline.
# usage: tools/bench_configs.sh TAG
tag=${1:?tag}
S=tools/gpu_step.sh
# (6 steps: the continuous lanes overlap step i + 1's prefill with step i's
# decode from the second step on)
for c in c2 c3 c4; do
  $S 600 ${tag}_bench_$c.log python -u bench.py --config $c --steps 6 --warmup 1; rc=$?
  [ $rc = 99 ] && exit 1
  grep '^{' gpurun_out/${tag}_bench_$c.log > gpurun_out/${tag}_bench_$c.json || true
done
exit 0
