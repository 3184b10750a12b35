#!/bin/bash
# Kernel traces of the config 4 step (auto: rating, then the MFMA kernel) and the forced
# k = 8 merge step on one GPU (rocprofv3 --kernel-trace --stats), summarised per kernel.
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/profr
run() {  # run NAME ARGS...
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/profr/$name" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" "$@" > "$ROOT/gpurun_out/profr/$name.log" 2>&1) \
      || { echo "!! $name"; tail -20 "$ROOT/gpurun_out/profr/$name.log"; exit 1; }
  f=$(ls "$ROOT"/gpurun_out/profr/$name/*/run_kernel_trace.csv "$ROOT"/gpurun_out/profr/$name/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/prof_summary.py "$f" ${TAIL:-30} > gpurun_out/profr/$name.txt
  echo "== $name"; head -16 gpurun_out/profr/$name.txt
}
run config4_auto --config 4 --steps 4 --warmup 1
TAIL=60 run merge_k8_forced --force-merge --merges-per-step 8 --steps 4 --warmup 1
