#!/bin/bash
# PMC passes (issue / wait / VALU / MFMA / LDS counters, one rocprofv3 run
# per counter group) over any lab command, for the kernels matching REGEX;
# prints the per-dispatch means per kernel.
# usage: tools/kernel_pmc.sh TAG REGEX python3 tools/<lab>.py [args]
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}; rx=${2:?regex}; shift 2
out=gpurun_out/$tag
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS"
for p in p1 p2; do
  case $p in p1) C=$P1;; p2) C=$P2;; esac
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$rx" --output-format csv \
      -d $out/$p -o $p -- "$@" > $out/$p.log 2>&1 || { tail -5 $out/$p.log; exit 1; }
  f=$(find $out/$p -name '*counter_collection.csv' | head -1); cp "$f" $out/$p.csv; rm -rf $out/$p
done
python3 - "$out" <<'PY'
import csv, sys, collections, re
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2"):
  for r in csv.DictReader(open(f"{out}/{p}.csv")):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[-60:]
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
  print(k)
  for c, v in sorted(d.items()):
    print(f"   {c:28s} mean/dispatch {sum(v)/len(v):.5g}  (n={len(v)})")
PY
