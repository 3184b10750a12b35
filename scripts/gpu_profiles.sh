#!/bin/bash
# Kernel-trace stats of the headline bench (config 2) and of config 4 (MFMA telemetry).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out/prof2 gpurun_out/prof4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof2 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 2 > $ROOT/gpurun_out/prof2/bench.log 2>&1 || { tail -5 $ROOT/gpurun_out/prof2/bench.log; exit 1; }
tail -1 $ROOT/gpurun_out/prof2/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof4 -o run --output-format csv -- python3 $ROOT/bench.py --config 4 --steps 5 --warmup 2 > $ROOT/gpurun_out/prof4/bench.log 2>&1 || { tail -5 $ROOT/gpurun_out/prof4/bench.log; exit 1; }
tail -1 $ROOT/gpurun_out/prof4/bench.log | cut -c1-200
