#!/bin/bash
# Prepass placement at the per-launch grid (round 5): the defaults against a serial prepass and
# tail-point sweeps (config 5: 1v1-3v3 kernels compiled for 4 waves per SIMD); gpurun_out/place5/
set -o pipefail
mkdir -p gpurun_out/place5
for r in 1 2; do
  for spec in ${PLACE_SPECS:-"5:default" "5:serial" "5:0" "5:0.05" "5:0.1" "2:default" "4:default"}; do
    c=${spec%%:*}; v=${spec#*:}
    e="X=0"; [ $v = serial ] && e="ANA_PREPASS_SERIAL=1"
    case $v in 0*) e="ANA_PREPASS_AT=$v";; esac
    env $e timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/place5/c${c}_${v}_$r.log 2>&1 || exit 1
    echo "config $c $v round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/place5/c${c}_${v}_$r.log)"
  done
done
