#!/bin/bash
# HBM traffic of the bench's dominant kernel from PMC counters, as the
# MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE in separate passes
# (one bench step each), HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB units;
# gfx950 FETCH_SIZE counts half of a wide streaming read).
# usage: tools/pmc_traffic.sh TAG REGEX   -> gpurun_out/TAG/pmc_*.csv
set -o pipefail
export TMPDIR=/tmp
# (round 4 ran these passes with CADENCE_SYNC_H2D=1 after rocprofv3's PMC
# mode crashed in hipEventRecord; round 5 runs the bench's default path:
# the crash did not reproduce -- DESIGN.md, "The rocprofv3 PMC crash")
tag=${1:?tag}; rx=${2:?regex}
out=gpurun_out/$tag
mkdir -p $out
export PYTHONFAULTHANDLER=1
for c in FETCH_SIZE WRITE_SIZE; do
  # the library map of each pass's process, for resolving a crash backtrace
  export CADENCE_DUMP_MAPS=$out/pmc_${c}_maps.txt
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$rx" --output-format csv \
      -d $out/pmc_$c -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
      --no-kernel-timing > $out/pmc_$c.log 2>&1 || { tail -20 $out/pmc_$c.log; exit 1; }
  f=$(find $out/pmc_$c -name '*counter_collection.csv' | head -1)
  cp "$f" $out/pmc_$c.csv
  rm -rf $out/pmc_$c
done
ls -la $out
