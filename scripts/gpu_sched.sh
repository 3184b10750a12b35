#!/bin/bash
# Schedule-prepass change: GPU tests, then bench (overlapped / serial) + standalone timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do echo "== bench serial=$v"; ANA_PREPASS_SERIAL=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --check > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log; done
timeout -k 10 300 python scripts/tune_rate.py --rounds 3 --blocks 512 > gpurun_out/tune.log 2>&1; tail -2 gpurun_out/tune.log
