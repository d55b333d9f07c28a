#!/bin/bash
# Continuous lanes with the asynchronous (default) vs blocking
# (CADENCE_SYNC_H2D=1) prompt copy at a rank's N = 8 load, C3 and C2.
# usage: tools/sync_h2d_ab.sh TAG
tag=${1:?tag}
export TMPDIR=/tmp
for cfg in "n8|--global-batch 32 --steps 16" "c3|--config c3 --steps 8" "c2|--config c2 --steps 6"; do
  name=${cfg%%|*}; args=${cfg#*|}
  for v in async sync; do
    envs=""; [ $v = sync ] && envs="CADENCE_SYNC_H2D=1"
    env $envs timeout -k 10 300 python bench.py $args --warmup 1 --no-cpu-baseline \
      --no-kernel-timing > gpurun_out/${tag}_${name}_$v.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/${tag}_${name}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name $v', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_enqueue_ms_per_step'])"
  done
done
