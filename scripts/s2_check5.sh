#!/bin/bash
# Round-3 session-2 GPU check 5: 8192-element sort tiles (512 threads) vs 4096:
# schedule parity under the variant library, then interleaved prepass/executor A/B.
set -o pipefail
mkdir -p gpurun_out/s2e
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2e/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2e/$name.log; exit $rc; fi
}
step sched_t512 600 env ANA_NATIVE_LIB=ab/t512_C.so python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 \
    --timeout-method thread -k "schedule or radix or levels"
tail -2 gpurun_out/s2e/sched_t512.log
for r in 1 2 3; do
  for spec in cur: t512:ab/t512_C.so; do
    name=${spec%%:*}; lib=${spec#*:}
    step random_${name}_$r 300 env ANA_NATIVE_LIB=$lib python scripts/tune_rate.py --pattern random --rounds 2 --local 1 --diag 0
    echo "$name $r $(grep -h '^round' gpurun_out/s2e/random_${name}_$r.log | sed -E 's/.*schedule +([0-9.]+) ms rate +([0-9.]+) ms.*/sched \1 rate \2 |/' | tr '\n' ' ')"
  done
done
