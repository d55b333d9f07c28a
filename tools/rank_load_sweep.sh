#!/bin/bash
# A rank's load at N = 1, 2, 4, 8 (global batch 256 / N on one GPU) under an
# RCCL process group of one rank (CADENCE_DIST_FORCE=1, torch.distributed.run,
# as the driver's multi-GPU runs), with and without the continuous lanes.
# usage: tools/rank_load_sweep.sh TAG [STEPS]
tag=${1:?tag}; steps=${2:-6}
export TMPDIR=/tmp CADENCE_DIST_FORCE=1
port=29700
for gb in 256 128 64 32; do
  for mode in cont nocont; do
    port=$((port + 1))
    extra=""; [ $mode = nocont ] && extra="--no-continuous"
    timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --global-batch $gb \
      --steps $steps --warmup 1 --no-cpu-baseline --no-kernel-timing $extra \
      > gpurun_out/${tag}_gb${gb}_$mode.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/${tag}_gb${gb}_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gb $gb $mode', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['generated_tokens_checksum'])"
  done
done
