#!/bin/bash
# Round-3 session-2 GPU check 3: the DP step with the next prepass beside the merge
# (engine.py merge_side): forced merges on one GPU at k = 1 / 8, a plain k = 1 step,
# and the 2-rank gloo rehearsal of the spawn path.
set -o pipefail
mkdir -p gpurun_out/s2c
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2c/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2c/$name.log; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -2 gpurun_out/s2c/tests.log
for r in 1 2; do
  for k in 1 8; do
    step merge_k${k}_$r 300 python bench.py --steps 20 --warmup 3 --merges-per-step $k --force-merge
    echo "force-merge k=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2c/merge_k${k}_$r.log) $(grep -o '"merge_ms": {[^}]*}' gpurun_out/s2c/merge_k${k}_$r.log)"
  done
  step plain_$r 300 python bench.py --steps 20 --warmup 3
  echo "plain $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2c/plain_$r.log)"
done
step gloo2 600 env ANA_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2
tail -1 gpurun_out/s2c/gloo2.log | cut -c1-600
# bench timeline: gaps between the prepass and the executor launch
mkdir -p gpurun_out/s2c/prof
ROOT=$(pwd); (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/s2c/prof" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/s2c/prof.log" 2>&1) \
  || { echo "!! prof"; tail -20 gpurun_out/s2c/prof.log; exit 1; }
f=$(find gpurun_out/s2c/prof -name run_kernel_trace.csv | head -1)
python3 scripts/prof_summary.py "$f" 40 > gpurun_out/s2c/prof_summary.txt
head -16 gpurun_out/s2c/prof_summary.txt
