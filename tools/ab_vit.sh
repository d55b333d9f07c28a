set -o pipefail
L=cadence-gemma_amd/cadence
cp $L/libcadence_hip.so /tmp/cur.so
for v in head batch occ4; do
  cp $L/_ab/lib_$v.so $L/libcadence_hip.so
  echo "== $v"
  timeout -k 10 120 python -u tools/vit_attn_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -q -k vit_attention --timeout 60 2>&1 | tail -1 || exit 1
done
cp /tmp/cur.so $L/libcadence_hip.so
