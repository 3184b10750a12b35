#!/bin/bash
# Tail-overlap threshold sweep (ANA_PREPASS_AT) on the bench, after the GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for at in ${ATS:-0 0.6 0.8 0.9 0.97 0.6 0.8 0.9}; do
  ANA_PREPASS_AT=$at timeout -k 10 200 python bench.py --steps 10 --warmup 3 --check > gpurun_out/tail.log 2>&1 || { tail -5 gpurun_out/tail.log; exit 1; }
  echo "at=$at $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tail.log)"
done
