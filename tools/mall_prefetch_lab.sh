#!/bin/bash
# Builds tools/mall_prefetch_lab (cross-launch weight prefetch, pure reads) on the CPU box.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mall_prefetch_lab.hip -o tools/mall_prefetch_lab
