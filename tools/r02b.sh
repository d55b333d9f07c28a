#!/bin/bash
S=tools/gpu_step.sh
$S 300 r02b_scan_eos.log python -u -m pytest tests/test_kernels_gpu.py -k scan tests/test_sampler_eos_gpu.py -x -v --timeout 120 --timeout-method thread; [ $? = 99 ] && exit 1
$S 120 r02b_scan_micro.log python -u tools/scan_micro.py; [ $? = 99 ] && exit 1
cat gpurun_out/r02b_scan_micro.log
$S 700 r02b_full.log python -u -m pytest tests/test_full_size_gpu.py -v -s --timeout 300 --timeout-method thread; [ $? = 99 ] && exit 1
grep -E "PASS|FAIL|Error|^E |^(c1|c2|c3|c4|p0|bench224) " gpurun_out/r02b_full.log | head -40
