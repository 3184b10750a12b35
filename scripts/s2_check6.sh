#!/bin/bash
# Round-3 session-2 GPU check 6: DP step placement (k = 8 forced merges): serial prepass
# beside the merge (default) vs tail-overlapped prepass at several start points.
set -o pipefail
mkdir -p gpurun_out/s2f
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/s2f/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -30 gpurun_out/s2f/$name.log; exit $rc; fi
}
for r in 1 2; do
  step serial_$r 300 python bench.py --steps 20 --warmup 3 --merges-per-step 8 --force-merge
  echo "serial $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2f/serial_$r.log)"
  for at in 0.5 0.7 0.9; do
    step tail${at}_$r 300 env ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$at python bench.py --steps 20 --warmup 3 --merges-per-step 8 --force-merge
    echo "tail $at $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2f/tail${at}_$r.log)"
  done
  step nomerge_$r 300 python bench.py --steps 20 --warmup 3 --merges-per-step 8
  echo "k8 no merge $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2f/nomerge_$r.log)"
  step plain_$r 300 python bench.py --steps 20 --warmup 3
  echo "plain $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2f/plain_$r.log)"
done
