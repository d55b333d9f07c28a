#!/bin/bash
# Multi-rank rehearsal of the bench's data-parallel path on a one-GPU box:
# torchrun with N ranks that all map onto cuda:0 (distributed.local_device_index)
# over the gloo backend (RCCL refuses two ranks on one GPU).  Checks launch,
# sharding (global batch 256 split over the ranks), the token all-gather, the
# max-over-ranks timing and rank 0's JSON line; not a scaling measurement.
# usage: tools/dp_rehearsal.sh TAG [N]
tag=${1:?tag}; n=${2:-2}
export TMPDIR=/tmp CADENCE_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $n --steps 2 --warmup 1 \
  --no-cpu-baseline --no-kernel-timing > gpurun_out/${tag}_dp$n.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/${tag}_dp$n.log | tail -5 | cut -c1-400
exit $rc
