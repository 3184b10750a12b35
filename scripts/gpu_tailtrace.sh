#!/bin/bash
# Kernel timeline of the bench with the tail overlap (rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ANA_PREPASS_AT=${AT:-0.8} timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/tprof -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 > $ROOT/gpurun_out/tprof.log 2>&1; rc=$?
tail -1 $ROOT/gpurun_out/tprof.log; exit $rc
