#!/bin/bash
S=tools/gpu_step.sh
$S 300 r02d_scan.log python -u -m pytest tests/test_kernels_gpu.py -k scan -x -v --timeout 120 --timeout-method thread; [ $? = 99 ] && exit 1
$S 120 r02d_scan_micro.log python -u tools/scan_micro.py; [ $? = 99 ] && exit 1
cat gpurun_out/r02d_scan_micro.log
$S 700 r02d_full.log python -u -m pytest tests/test_full_size_gpu.py -v -s --timeout 300 --timeout-method thread; [ $? = 99 ] && exit 1
grep -E "^E |PASSED|FAILED" gpurun_out/r02d_full.log | head -40
$S 400 r02d_bench.log python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline; [ $? = 99 ] && exit 1
grep '^{' gpurun_out/r02d_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms/step',d['ms_per_step'],d['ms_per_step_median'],'prefill_ms',d['prefill_ms'], d['roofline_decode'])"
