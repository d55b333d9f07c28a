#!/bin/bash
# PMC passes over tools/vit_one.py (one ViT attention shape): SQ issue /
# wait / MFMA-busy counters and LDS, one pass each.
# usage: tools/vit_pmc.sh TAG   (env SHAPE / ENGINE passed through)
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 120 python3 -u tools/vit_one.py > $out/plain.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "vit_" --output-format csv -d $out/p1 -o p1 -- python3 tools/vit_one.py > $out/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --kernel-include-regex "vit_" --output-format csv -d $out/p2 -o p2 -- python3 tools/vit_one.py > $out/p2.log 2>&1 || exit 1
for p in p1 p2; do f=$(find $out/$p -name '*counter_collection.csv' | head -1); cp "$f" $out/$p.csv; rm -rf $out/$p; done
python3 - "$out" <<'PY'
import csv, sys, collections
out = sys.argv[1]
for p in ("p1", "p2"):
  acc = collections.defaultdict(list)
  for r in csv.DictReader(open(f"{out}/{p}.csv")):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
  for k, v in sorted(acc.items()):
    print(f"{p} {k:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
cat $out/plain.log
