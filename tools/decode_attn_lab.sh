#!/bin/bash
# Decode attention split plan sweep (CADENCE_DEC_F workgroups per batch,
# CADENCE_DEC_CMIN fewest keys per range) on tools/decode_attn_micro.py.
# The two knobs were environment variables of the lab build of commit
# b29c322 only (the shipped library reads no environment: F = 256,
# kDecodeMinRange = 64 are compile-time constants of attention.hip).
# usage: tools/decode_attn_lab.sh TAG
set -o pipefail
tag=${1:?tag}
log=gpurun_out/${tag}_dec_lab.log
: > $log
for f in 256 512 1024; do for c in 16 64 128; do
  echo "== F=$f CMIN=$c" >> $log
  CADENCE_DEC_F=$f CADENCE_DEC_CMIN=$c timeout -k 10 120 python -u tools/decode_attn_micro.py >> $log 2>&1 || exit 1
done; done
cat $log | grep -v amdgpu.ids
