#!/bin/bash
# SURVEY §5 sanitizer row: the C-ABI's host code (launch plans, workspace
# and plan queries, contract checks, the batched-copy descriptor checks)
# under AddressSanitizer, CPU only: builds build/asan/libcadence_hip_asan.so
# (make asan: -Xarch_host -fsanitize=address) and runs the C-ABI tests that
# call it without a GPU (tests/test_abi_api.py) with the ASan runtime
# preloaded.  Python's own allocations are not leak-checked.
# usage: tools/asan_host.sh [pytest args]
set -e -o pipefail
cd "$(dirname "$0")/.."
make -C cadence-gemma_amd asan -j8 >/dev/null
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LIB=$PWD/cadence-gemma_amd/build/asan/libcadence_hip_asan.so
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 CADENCE_LIB_PATH=$LIB \
  python -m pytest tests/test_abi_api.py -q -m "not gpu" -p no:cacheprovider "$@"
