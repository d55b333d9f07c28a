#!/bin/bash
S=tools/gpu_step.sh
$S 120 r02j_dbg.log python -u tools/attn_debug.py; [ $? = 99 ] && exit 1
cat gpurun_out/r02j_dbg.log | grep -v amdgpu.ids
$S 300 r02j_attn.log python -u -m pytest tests/test_kernels_gpu.py -k "local_attention or vit_attention" -v --timeout 120 --timeout-method thread; rc=$?; [ $rc != 0 ] && exit 1
$S 120 r02j_attn_micro.log python -u tools/attn_micro.py; [ $? = 99 ] && exit 1
$S 120 r02j_vit_micro.log python -u tools/vit_attn_micro.py; [ $? = 99 ] && exit 1
cat gpurun_out/r02j_attn_micro.log gpurun_out/r02j_vit_micro.log | grep -v amdgpu.ids
exit 0
