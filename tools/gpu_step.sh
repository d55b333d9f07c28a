#!/bin/bash
# Runs one GPU step under its own time limit, logging to gpurun_out/<log>.
# usage: tools/gpu_step.sh SECONDS LOG cmd...   exit status: the step's, and
# a fault / abort / timeout (124 134 137 139) is reported so the caller stops.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "[$log] rc $rc"
tail -4 "gpurun_out/$log"
case $rc in 124|134|137|139) echo "[$log] fault/timeout: stopping"; exit 99;; esac
exit $rc
