#!/bin/bash
# Executor grid A/B (round 5): the per-launch choice (ops/rate.py launch_blocks) against a fixed 512,
# configs 2-5 and the forced k = 8 DP step, interleaved; output under gpurun_out/grid3/
set -o pipefail
mkdir -p gpurun_out/grid3
for r in 1 2; do
  for b in auto 512; do
    e=""; [ $b != auto ] && e="ANA_RATE_BLOCKS=$b"
    for c in 2 3 4 5; do
      env $e timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/grid3/c${c}_${b}_$r.log 2>&1 || exit 1
      echo "config $c blocks $b round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/grid3/c${c}_${b}_$r.log)"
    done
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 > gpurun_out/grid3/dp8_${b}_$r.log 2>&1 || exit 1
    echo "forced k=8 blocks $b round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/grid3/dp8_${b}_$r.log)"
  done
done
