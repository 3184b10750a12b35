#!/bin/bash
# Round-3 session-2 GPU check 7: (a) prepass tail-overlap start for the plain config 2
# step and for k = 8 forced merges; (b) one-lane-per-row telemetry (ANA_TELE_IMPL=2):
# oracle tests, kernel timing vs MFMA, config 4 separate.
set -o pipefail
mkdir -p gpurun_out/s2g
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2g/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2g/$name.log; exit $rc; fi
}
step teletests 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "telemetry"
tail -2 gpurun_out/s2g/teletests.log
step tune_tele3 300 python scripts/tune_tele.py --variants impl1,impl2 --rounds 3
grep -h '^round' gpurun_out/s2g/tune_tele3.log | tail -2
step tune_tele5 300 python scripts/tune_tele.py --variants impl1,impl2 --rounds 3 --team-size 5 --matches 2000000
grep -h '^round' gpurun_out/s2g/tune_tele5.log | tail -2
for r in 1 2; do
  step plain_$r 300 python bench.py --steps 20 --warmup 3
  echo "plain serial $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2g/plain_$r.log)"
  for at in 0.85 0.9 0.95; do
    step plain_tail${at}_$r 300 env ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$at python bench.py --steps 20 --warmup 3
    echo "plain tail $at $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2g/plain_tail${at}_$r.log)"
  done
  for at in 0.9 0.95; do
    step k8_tail${at}_$r 300 env ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$at python bench.py --steps 20 --warmup 3 --merges-per-step 8 --force-merge
    echo "k8 forced tail $at $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2g/k8_tail${at}_$r.log)"
  done
  for impl in 1 2; do
    step c4_impl${impl}_$r 300 env ANA_TELE_IMPL=$impl python bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode separate
    echo "config4 separate impl$impl $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2g/c4_impl${impl}_$r.log)"
  done
done
