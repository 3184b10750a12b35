#!/bin/bash
# GPU check of everything new: kernel tests, the re-rate driver (config 5 shape on 1 GPU), bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== rerate ${RERATE_MATCHES:-1e8} matches / ${RERATE_PLAYERS:-1e7} players"
timeout -k 10 600 python -m analyzer_amd.runtime.rerate --matches ${RERATE_MATCHES:-1e8} --players ${RERATE_PLAYERS:-1e7} --window ${RERATE_WINDOW:-1.6e7} > gpurun_out/rerate.log 2>&1; rc=$?
tail -1 gpurun_out/rerate.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps 10 --warmup 3 --check > gpurun_out/bench.log 2>&1; rc=$?
tail -1 gpurun_out/bench.log; exit $rc
