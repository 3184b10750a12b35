#!/bin/bash
# Full GPU suite + micro-batch bench (3v3, 5v5) + config-2 bench, 1x MI355X.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_tests.log 2>&1 || { tail -30 gpurun_out/v_tests.log; exit 1; }
tail -1 gpurun_out/v_tests.log
for k in 3 5; do
  timeout -k 10 120 python scripts/bench_graph.py --batches 200 --team-size $k > gpurun_out/v_micro$k.log 2>&1 || { tail -20 gpurun_out/v_micro$k.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/v_micro$k.log
done
timeout -k 10 180 python bench.py > gpurun_out/v_bench.log 2>&1 || { tail -20 gpurun_out/v_bench.log; exit 1; }
grep metric gpurun_out/v_bench.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof -o v -- python scripts/bench_graph.py --batches 50 > gpurun_out/v_prof.log 2>&1 || { tail -20 gpurun_out/v_prof.log; exit 1; }
echo done
