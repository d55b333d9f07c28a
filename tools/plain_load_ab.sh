#!/bin/bash
# Plain (no process group) bench at a rank's N = 8 load and at N = 1, with and
# without the continuous lanes.  usage: tools/plain_load_ab.sh TAG
tag=${1:?tag}
export TMPDIR=/tmp
for cfg in "32 20" "256 5"; do
  set -- $cfg
  for mode in cont nocont; do
    extra=""; [ $mode = nocont ] && extra="--no-continuous"
    timeout -k 10 300 python bench.py --global-batch $1 --steps $2 --warmup 1 --no-cpu-baseline \
      --no-kernel-timing $extra > gpurun_out/${tag}_gb$1_$mode.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/${tag}_gb$1_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gb $1 $mode', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['generated_tokens_checksum'])"
  done
done
