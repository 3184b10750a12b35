#!/bin/bash
# Round-3 session-2 GPU check 2: full GPU suite on the pipelined inline telemetry +
# lane-per-track merge kernels; config 4 A/B; the 10-bit-digit prepass kernel split.
set -o pipefail
mkdir -p gpurun_out/s2b
ROOT=$(pwd)
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2b/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2b/$name.log; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -3 gpurun_out/s2b/tests.log
for mode in inline separate inline2 separate2; do
  case $mode in inline*) env="ANA_TELE_ROLE=-1"; tm=fused;; separate*) env="ANA_TELE_ROLE=2"; tm=separate;; esac
  step c4_$mode 300 env $env python bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode $tm
  echo "config4 $mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2b/c4_$mode.log)"
done
for rb in 8 10; do
  mkdir -p gpurun_out/s2b/prof_rb$rb
  (cd /tmp && ANA_SORT_RB=$rb timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/s2b/prof_rb$rb" \
      -o run --output-format csv -- python3 "$ROOT/scripts/tune_rate.py" --pattern random --rounds 2 \
      > "$ROOT/gpurun_out/s2b/prof_rb$rb.log" 2>&1) || { echo "!! prof rb$rb"; tail -20 gpurun_out/s2b/prof_rb$rb.log; exit 1; }
  f=$(ls gpurun_out/s2b/prof_rb$rb/*/run_kernel_trace.csv gpurun_out/s2b/prof_rb$rb/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/prof_summary.py "$f" 24 > gpurun_out/s2b/prof_rb$rb.txt
  head -14 gpurun_out/s2b/prof_rb$rb.txt
done
