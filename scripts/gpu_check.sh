#!/bin/bash
# GPU validation + measurement, one box call.  Each GPU step has its own time
# limit; a crash/abort/timeout ends the script (no further GPU work).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
stop_on_fault() {  # $1 = exit code; 0/1 (test failures) continue, anything else stops
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "GPU step failed hard (exit $1); stopping"; exit "$1"; fi
}
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -25 $OUT/pytest_gpu.log; stop_on_fault $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -5 $OUT/smoke.log; stop_on_fault $rc
echo "== bench"; date
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-5} --warmup 2 --check > $OUT/bench.log 2>&1; rc=$?
tail -5 $OUT/bench.log; stop_on_fault $rc
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3"; date
  ROOT=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 > $ROOT/$OUT/prof.log 2>&1); rc=$?
  tail -5 $OUT/prof.log; stop_on_fault $rc
  find $OUT/prof -name "*stats*" | head
fi
echo "== done"; date
