#!/bin/bash
# Prepass placement at the per-launch grid (round 5): the new defaults (tail overlap at 0.75 for a
# one-wave-per-SIMD launch) vs a serial prepass, and config 4's shared tail point; gpurun_out/place3/
set -o pipefail
mkdir -p gpurun_out/place3
for r in 1 2; do
  for spec in "2:default" "2:serial" "4:default" "4:0.4" "4:0.3" "3:default" "5:default"; do
    c=${spec%%:*}; v=${spec#*:}
    e=""; [ $v = serial ] && e="ANA_PREPASS_SERIAL=1"
    case $v in 0.*) e="ANA_TELE_TAIL_AT=$v";; esac
    env $e timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/place3/c${c}_${v}_$r.log 2>&1 || exit 1
    echo "config $c $v round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/place3/c${c}_${v}_$r.log)"
  done
done
