#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc; stopping"; exit $rc; fi
run() { echo "== $*"; timeout -k 10 300 python scripts/tune_rate.py --rounds 2 "$@" > gpurun_out/micro.log 2>&1; rc=$?; tail -1 gpurun_out/micro.log; cat gpurun_out/micro.log >> gpurun_out/micro_all.log; [ $rc -eq 0 ] || exit $rc; }
run --pattern serial --players 1000 --matches 20000 --blocks 8,512
run --pattern disjoint --players 6000000 --matches 1000000 --blocks 256,1024
run --pattern random --players 1000000 --matches 10000000 --blocks 256,512,1024
echo "== bench"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 --check > gpurun_out/bench.log 2>&1; rc=$?
tail -2 gpurun_out/bench.log; exit $rc
