#!/bin/bash
# Sweep the idle back-off of the dataflow executor (ANA_RATE_IDLE) on the bench stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 300 python scripts/tune_rate.py --rounds 2 "$@" > gpurun_out/micro.log 2>&1; rc=$?; tail -1 gpurun_out/micro.log; cat gpurun_out/micro.log >> gpurun_out/micro_all.log; [ $rc -eq 0 ] || exit $rc; }
run --pattern random --players 1000000 --matches 10000000 --blocks 512,1024 --idle ${IDLE:-1,4,8,32,128}
run --pattern serial --players 1000 --matches 20000 --blocks 512 --idle ${IDLE:-1,4,8,32,128}
