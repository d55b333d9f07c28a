#!/bin/bash
# Headline bench A/B on one box: default, --no-continuous, and the blocking
# host->device prompt copy (CADENCE_SYNC_H2D=1), two rounds interleaved.
# usage: tools/headline_ab.sh TAG [STEPS]
tag=${1:?tag}; steps=${2:-4}
export TMPDIR=/tmp
for r in 1 2; do
  for v in default nocont synch2d; do
    extra=""; envs=""
    [ $v = nocont ] && extra="--no-continuous"
    [ $v = synch2d ] && envs="CADENCE_SYNC_H2D=1"
    env $envs timeout -k 10 300 python bench.py --steps $steps --warmup 1 --no-cpu-baseline \
      $extra > gpurun_out/${tag}_${v}_$r.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/${tag}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $r', d['value'], d['ms_per_step'], d['roofline_decode']['avg_us'], d['roofline']['avg_us'], d['host_enqueue_ms_per_step'])"
  done
done
