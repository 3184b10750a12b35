#!/bin/bash
# Kernel timeline of bench config 4 (separate telemetry kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/c4prof -o run --output-format csv -- python3 $ROOT/bench.py --config 4 --telemetry-mode ${MODE:-separate} --steps 3 --warmup 1 > $ROOT/gpurun_out/c4prof.log 2>&1; rc=$?
tail -1 $ROOT/gpurun_out/c4prof.log | cut -c1-200; exit $rc
