#!/bin/bash
# Round-3 session-2 GPU check: inline telemetry (ANA_TELE_ROLE=-1) + lane-per-track
# merge kernels over base rows.  Tests first; every GPU step bounded; stop at the
# first failure.
set -o pipefail
mkdir -p gpurun_out/s2
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2/$name.log; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "telemetry or sweep or rccl or merge"
tail -3 gpurun_out/s2/tests.log
step merge_micro 300 python scripts/merge_micro.py --players 1e6,1e7
tail -4 gpurun_out/s2/merge_micro.log
for mode in inline separate role2 inline2 separate2; do
  case $mode in inline*) env="ANA_TELE_ROLE=-1"; tm=fused;; separate*) env="ANA_TELE_ROLE=2"; tm=separate;; role2) env="ANA_TELE_ROLE=2"; tm=fused;; esac
  step c4_$mode 300 env $env python bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode $tm
  echo "config4 $mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2/c4_$mode.log)"
done
for k in 1 8; do
  step merge_k$k 300 python bench.py --steps 20 --warmup 3 --merges-per-step $k --force-merge
  echo "force-merge k=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2/merge_k$k.log) $(grep -o '"merge_ms": {[^}]*}' gpurun_out/s2/merge_k$k.log)"
done
