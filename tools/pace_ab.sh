#!/bin/bash
# Lane pacing A/B (CADENCE_LANE_PACE): N = 1 headline and C3, two rounds.
tag=${1:?tag}
export TMPDIR=/tmp
for r in 1 2; do
  for v in 1 0; do
    CADENCE_LANE_PACE=$v timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline \
      --no-kernel-timing > gpurun_out/${tag}_n1_pace${v}_$r.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/${tag}_n1_pace${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n1 pace $v', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
    CADENCE_LANE_PACE=$v timeout -k 10 300 python bench.py --config c3 --steps 8 --warmup 1 --no-cpu-baseline \
      --no-kernel-timing > gpurun_out/${tag}_c3_pace${v}_$r.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/${tag}_c3_pace${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 pace $v', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
  done
done
