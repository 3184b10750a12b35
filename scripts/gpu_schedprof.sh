#!/bin/bash
# Schedule GPU tests + per-kernel times of the schedule prepass alone (rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "schedule or radix" > gpurun_out/pytest_sched.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sched.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/sprof -o run --output-format csv -- python3 $ROOT/scripts/sched_time.py > $ROOT/gpurun_out/sprof.log 2>&1; rc=$?
tail -1 $ROOT/gpurun_out/sprof.log; exit $rc
