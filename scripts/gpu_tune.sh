#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "hard failure $rc"; exit $rc; fi
echo "== tune"; timeout -k 10 600 python scripts/tune_rate.py --rounds 2 ${TUNE_ARGS} > gpurun_out/tune.log 2>&1; rc=$?
tail -15 gpurun_out/tune.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 --check > gpurun_out/bench.log 2>&1; rc=$?
tail -3 gpurun_out/bench.log; exit $rc
