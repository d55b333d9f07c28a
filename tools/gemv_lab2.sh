#!/bin/bash
# Builds tools/gemv_lab2 (decode residual-projection variants, cold weights) on the CPU box.
set -e
cd "$(dirname "$0")/.."
make -s -C cadence-gemma_amd build/norm.o >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/gemv_lab2.hip -o /tmp/gemv_lab2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/gemv_lab2.o cadence-gemma_amd/build/norm.o -o tools/gemv_lab2
