#!/bin/bash
# Round-3 session-2 GPU check 4: schedule last pass with a run-end table (no digit
# offsets) -- schedule parity tests, then the prepass split and the config 2 step.
set -o pipefail
mkdir -p gpurun_out/s2d
ROOT=$(pwd)
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2d/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2d/$name.log; exit $rc; fi
}
step sched 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "schedule or levels or radix"
tail -2 gpurun_out/s2d/sched.log
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -2 gpurun_out/s2d/tests.log
for r in 1 2; do
  for runs in 1 0; do
    step bench_runs${runs}_$r 300 env ANA_SCHED_RUNS=$runs python bench.py --steps 20 --warmup 3
    echo "runs=$runs $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2d/bench_runs${runs}_$r.log)"
  done
done
mkdir -p gpurun_out/s2d/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/s2d/prof" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/s2d/prof.log" 2>&1) \
  || { echo "!! prof"; tail -20 gpurun_out/s2d/prof.log; exit 1; }
f=$(find gpurun_out/s2d/prof -name run_kernel_trace.csv | head -1)
python3 scripts/prof_summary.py "$f" 16 > gpurun_out/s2d/prof_summary.txt
cat gpurun_out/s2d/prof_summary.txt
