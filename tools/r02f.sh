#!/bin/bash
S=tools/gpu_step.sh
$S 120 r02f_scan_micro.log python -u tools/scan_micro.py; [ $? = 99 ] && exit 1
cat gpurun_out/r02f_scan_micro.log
