#!/bin/bash
# PMC passes over vit_fa32_kernel (the lab build, 20 launches of one shape),
# one counter set per rocprofv3 run (slot limits: MI355X_MICROARCH.md).
# usage: tools/vit_fa32_pmc.sh TAG SHAPE [LAB]
set -o pipefail
export TMPDIR=/tmp
tag=${1:?tag}; shape=${2:-dino336}; lab=${3:-0}
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 tools/vit_fa32_lab.py --pmc $shape $lab > $out/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    if "fa32" not in r.get("Kernel_Name", ""):
      continue
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
  v = agg[k]
  print(f"{k:28s} per-dispatch mean {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
