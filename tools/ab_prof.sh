#!/bin/bash
# Per-kernel A/B of prebuilt libraries (cadence/_ab/lib_<name>.so): a short
# bench under rocprofv3 --kernel-trace --stats per library, then the average
# duration of every kernel matching REGEX.
# usage: tools/ab_prof.sh REGEX name1 name2 ...
set -o pipefail
export TMPDIR=/tmp
L=cadence-gemma_amd/cadence
rx=$1; shift
cp $L/libcadence_hip.so /tmp/cur.so
for v in "$@"; do
  cp $L/_ab/lib_$v.so $L/libcadence_hip.so
  d=gpurun_out/abprof_$v
  rm -rf $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $d.log 2>&1 \
      || { cp /tmp/cur.so $L/libcadence_hip.so; tail -5 $d.log; exit 1; }
  f=$(find $d -name '*kernel_stats.csv' | head -1)
  echo "== $v  $(grep -o '"value": [0-9.]*' $d.log)"
  python3 - "$f" "$rx" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
  if re.search(sys.argv[2], r["Name"]):
    print(f'{float(r["AverageNs"]) / 1e3:9.2f} us {int(r["Calls"]):7d}  {r["Name"][:110]}')
PY
  rm -rf $d
done
cp /tmp/cur.so $L/libcadence_hip.so
