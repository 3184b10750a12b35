#!/bin/bash
# schedule sort with non-temporal key/value/link traffic: A/B on the bench (co-running prepass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sort
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "schedule" > gpurun_out/sort/pytest.log 2>&1 || { tail -30 gpurun_out/sort/pytest.log; exit 1; }
ANA_SORT_NT=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "schedule" > gpurun_out/sort/pytest_nt.log 2>&1 || { tail -30 gpurun_out/sort/pytest_nt.log; exit 1; }
tail -1 gpurun_out/sort/pytest_nt.log
for nt in 0 1; do
  ANA_SORT_NT=$nt timeout -k 10 300 python scripts/tune_rate.py --rounds 2 --blocks 512 > gpurun_out/sort/tune_nt$nt.log 2>&1 || exit 1
  echo "nt=$nt $(grep -o '"schedule_ms_min": [0-9.]*, "rate_ms_min": [0-9.]*' gpurun_out/sort/tune_nt$nt.log)"
done
for rep in 1 2 3; do for nt in 0 1; do
  ANA_SORT_NT=$nt timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/sort/b.log 2>&1 || { tail -5 gpurun_out/sort/b.log; exit 1; }
  echo "bench nt=$nt $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sort/b.log)"
done; done
