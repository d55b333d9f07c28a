#!/bin/bash
# A rank's N = 8 load (global batch 32, one micro-batch per step) with and
# without the continuous lanes, plain and under an RCCL process group of
# one rank (CADENCE_DIST_FORCE=1), 20 steps each, two rounds interleaved.
# usage: tools/n8_load_ab.sh TAG
tag=${1:?tag}
export TMPDIR=/tmp
run() {  # name, extra args...
  local name=$1; shift
  timeout -k 10 200 "$@" --global-batch 32 --steps 20 --warmup 2 --no-cpu-baseline \
    --no-kernel-timing > gpurun_out/${tag}_$name.log 2>&1 || return 1
  grep '^{"metric"' gpurun_out/${tag}_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['generated_tokens_checksum'])"
}
port=29600
for r in 1 2; do
  run plain_cont_$r python bench.py || exit 1
  run plain_nocont_$r python bench.py --no-continuous || exit 1
  port=$((port + 1))
  CADENCE_DIST_FORCE=1 run rccl_cont_$r python -m torch.distributed.run --nnodes 1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 || exit 1
  port=$((port + 1))
  CADENCE_DIST_FORCE=1 run rccl_nocont_$r python -m torch.distributed.run --nnodes 1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 \
    --no-continuous || exit 1
done
