# A/B two prebuilt libraries (cadence/_ab/lib_<name>.so) on one command.
# usage: tools/ab_lib.sh "cmd ..." name1 name2 ...
set -o pipefail
L=cadence-gemma_amd/cadence
cmd=$1; shift
cp $L/libcadence_hip.so /tmp/cur.so
for v in "$@"; do
  cp $L/_ab/lib_$v.so $L/libcadence_hip.so
  echo "== $v"
  timeout -k 10 300 bash -c "$cmd" 2>&1 | grep -v amdgpu.ids || { cp /tmp/cur.so $L/libcadence_hip.so; exit 1; }
done
cp /tmp/cur.so $L/libcadence_hip.so
