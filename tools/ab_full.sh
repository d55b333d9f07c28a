set -o pipefail
L=cadence-gemma_amd/cadence
cp $L/libcadence_hip.so /tmp/cur.so
for v in head new head new; do
  cp $L/_ab/lib_$v.so $L/libcadence_hip.so
  echo "== $v"
  timeout -k 10 200 python -u -m pytest tests/test_full_size_gpu.py -q -k bench224 -s --timeout 150 2>&1 | grep -o '"features_rel_l2\[0\]": [0-9.]*\|"prefill\[0\]": {[^}]*}\|passed\|failed' | head -4
done
cp /tmp/cur.so $L/libcadence_hip.so
