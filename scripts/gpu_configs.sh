#!/bin/bash
# BASELINE configs on one GPU: pytest -m gpu, then bench configs 2, 3, 4 (fused vs separate telemetry).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
b() { echo "== bench $*"; timeout -k 10 600 python bench.py --steps 10 --warmup 3 --check "$@" > gpurun_out/bench_cfg.log 2>&1; rc=$?; tail -1 gpurun_out/bench_cfg.log; cat gpurun_out/bench_cfg.log >> gpurun_out/bench_configs.log; [ $rc -eq 0 ] || exit $rc; }
b --config 2
b --config 3
b --config 4 --telemetry-mode fused
b --config 4 --telemetry-mode separate
