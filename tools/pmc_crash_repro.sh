#!/bin/bash
# The rocprofv3 PMC-mode crash: the plain-torch reproducer without and with
# the profiler, then (if it did not crash) the bench's default path (the
# asynchronous pinned prompt copies) under one PMC pass.  A segfault ends
# the script (nothing more runs on the GPU after it).
# usage: tools/pmc_crash_repro.sh TAG [MODE]
tag=${1:?tag}; mode=${2:-full}
S=tools/gpu_step.sh
export PYTHONFAULTHANDLER=1
$S 120 ${tag}_repro_plain.log python -u tools/pmc_crash_repro.py $mode || exit 1
$S 120 ${tag}_repro_pmc.log rocprofv3 --pmc FETCH_SIZE --output-format csv \
   -d gpurun_out/${tag}_repro -o run -- python3 -u tools/pmc_crash_repro.py $mode || exit 1
export CADENCE_DUMP_MAPS=gpurun_out/${tag}_bench_pmc_maps.txt
$S 240 ${tag}_bench_pmc.log rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_w4 \
   --output-format csv -d gpurun_out/${tag}_bench_pmc -o run -- python3 -u bench.py \
   --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing || exit 1
