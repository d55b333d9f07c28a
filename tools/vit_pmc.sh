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
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY TA_BUFFER_READ_LDS_WAVEFRONTS"
P3="SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD"
for p in p1 p2 p3; do
  case $p in p1) C=$P1;; p2) C=$P2;; p3) C=$P3;; esac
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "vit_" --output-format csv -d $out/$p -o $p -- python3 tools/vit_one.py > $out/$p.log 2>&1 || exit 1
done
for p in p1 p2 p3; do f=$(find $out/$p -name '*counter_collection.csv' | head -1); cp "$f" $out/$p.csv; rm -rf $out/$p; done
python3 - "$out" <<'PY'
import csv, sys, collections
out = sys.argv[1]
for p in ("p1", "p2", "p3"):
  acc = collections.defaultdict(list)
  for r in csv.DictReader(open(f"{out}/{p}.csv")):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
  for k, v in sorted(acc.items()):
    print(f"{p} {k:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
cat $out/plain.log
