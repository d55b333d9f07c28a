#!/bin/bash
# PMC traffic of the decode kernels on the eager path (tools/decode_pmc.py):
# separate --pmc FETCH_SIZE / WRITE_SIZE passes, then the per-kernel summary.
# usage: tools/decode_pmc.sh TAG   -> gpurun_out/TAG/, gpurun_out/TAG_decode_pmc.json
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
rx='gemm_gated_pipe|gemm_stream|gemm_resid_pipe|decode_attn|gemm_skinny|rglru_step'
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$rx" --output-format csv \
      -d $out/pmc_$c -o run -- python3 tools/decode_pmc.py 4 > $out/pmc_$c.log 2>&1 \
      || { tail -20 $out/pmc_$c.log; exit 1; }
  f=$(find $out/pmc_$c -name '*counter_collection.csv' | head -1)
  cp "$f" $out/pmc_$c.csv
  rm -rf $out/pmc_$c
done
python3 tools/decode_pmc.py --summary $out gpurun_out/${tag}_decode_pmc.json
