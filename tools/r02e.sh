#!/bin/bash
S=tools/gpu_step.sh
$S 300 r02e_scan.log python -u -m pytest tests/test_kernels_gpu.py -k scan -x -v --timeout 120 --timeout-method thread; [ $? = 99 ] && exit 1
$S 120 r02e_scan_micro.log python -u tools/scan_micro.py; [ $? = 99 ] && exit 1
cat gpurun_out/r02e_scan_micro.log
