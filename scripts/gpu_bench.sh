#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== bench"; timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 --check ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  ROOT=$(pwd)
  echo "== rocprofv3 kernel trace"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 > $ROOT/gpurun_out/prof.log 2>&1); rc=$?
  tail -2 gpurun_out/prof.log; exit $rc
fi
