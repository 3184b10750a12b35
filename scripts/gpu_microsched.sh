#!/bin/bash
# Micro-batch schedule A/B: LDS hash-list kernel (default) vs bitonic sort (ANA_SCHED_SMALL=bitonic).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "schedule or graph or device_matches" > gpurun_out/ms_tests.log 2>&1 || { tail -30 gpurun_out/ms_tests.log; exit 1; }
tail -2 gpurun_out/ms_tests.log
for v in hash bitonic; do
  echo "## $v"
  ANA_SCHED_SMALL=$v timeout -k 10 120 python scripts/bench_graph.py --batches 200 > gpurun_out/ms_$v.log 2>&1 || { tail -20 gpurun_out/ms_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ms_$v.log
  ANA_SCHED_SMALL=$v timeout -k 10 120 python scripts/bench_graph.py --batches 200 --team-size 5 > gpurun_out/ms5_$v.log 2>&1 || { tail -20 gpurun_out/ms5_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ms5_$v.log
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/msprof -o ms -- python scripts/bench_graph.py --batches 50 > gpurun_out/ms_prof.log 2>&1 || { tail -20 gpurun_out/ms_prof.log; exit 1; }
echo done
