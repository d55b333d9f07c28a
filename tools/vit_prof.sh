#!/bin/bash
# Vision phase alone: 2-stream vs 1-stream wall time, then rocprofv3 stats of
# the one-stream pass.  usage: tools/vit_prof.sh TAG [PX]
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}; px=${2:-224}
tools/gpu_step.sh 300 ${tag}_vit_phase.log python -u tools/vit_phase.py --px $px || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 tools/vit_phase.py --one-stream-only --px $px --reps 5 > gpurun_out/${tag}_vprof.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 30 > gpurun_out/${tag}_vit_kstats.txt
rm -rf gpurun_out/prof_$tag
cat gpurun_out/${tag}_vit_kstats.txt
SHAPES=8352x3072x1024,8352x1024x1024,8352x4096x1024,8352x1024x4096,8192x3456x1152,8192x1152x1152,8192x4352x1152,8192x1152x4352 VS_TORCH=1 timeout -k 10 300 python -u tools/gemm_shapes.py > gpurun_out/${tag}_vit_shapes.log 2>&1 || exit 1
cat gpurun_out/${tag}_vit_shapes.log
