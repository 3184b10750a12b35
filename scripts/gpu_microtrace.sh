#!/bin/bash
# Kernel trace of the 500-match micro-batch path (eager + graph replay), 1x MI355X.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_graph.py --batches 200 > gpurun_out/micro_bench.log 2>&1 || { tail -20 gpurun_out/micro_bench.log; exit 1; }
cat gpurun_out/micro_bench.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/microprof -o micro -- python scripts/bench_graph.py --batches 50 > gpurun_out/micro_prof.log 2>&1 || { tail -20 gpurun_out/micro_prof.log; exit 1; }
find gpurun_out/microprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-220 | head -20
