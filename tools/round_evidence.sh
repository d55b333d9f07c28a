#!/bin/bash
# Round-end evidence in one GPU call: the GPU parity suite + smoke, the
# default bench line (with cpu_baseline) and a rocprofv3 --kernel-trace
# --stats run of the same command, then the C2 / C3 / C4 lines.
# usage: tools/round_evidence.sh TAG
tag=${1:?tag}
bash tools/gpu_suite.sh $tag || exit 1
bash tools/profile_round.sh $tag || exit 1
bash tools/bench_configs.sh $tag || exit 1
