#!/bin/bash
# schedule sort digit width A/B (ANA_SORT_RB=8 vs the 10-bit default for <= 2^20 players)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sort
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sort/pytest.log 2>&1 || { tail -30 gpurun_out/sort/pytest.log; exit 1; }
tail -1 gpurun_out/sort/pytest.log
for rb in 8 10; do
  ANA_SORT_RB=$rb timeout -k 10 300 python scripts/tune_rate.py --rounds 2 --blocks 512 > gpurun_out/sort/tune_$rb.log 2>&1 || { tail -5 gpurun_out/sort/tune_$rb.log; exit 1; }
  echo "rb=$rb $(grep -o '"schedule_ms_min": [0-9.]*, "rate_ms_min": [0-9.]*' gpurun_out/sort/tune_$rb.log)"
done
for rep in 1 2; do for rb in 8 10; do
  ANA_SORT_RB=$rb timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/sort/b.log 2>&1 || { tail -5 gpurun_out/sort/b.log; exit 1; }
  echo "bench rb=$rb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sort/b.log)"
done; done
