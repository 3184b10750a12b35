#!/bin/bash
# A/B: executor issue priority (ANA_RATE_DEBUG=8) x tail-overlap threshold.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do for dbg in 0 8; do for at in 0 0.7 0.85; do
  ANA_RATE_DEBUG=$dbg ANA_PREPASS_AT=$at timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/prio.log 2>&1 || { tail -5 gpurun_out/prio.log; exit 1; }
  echo "dbg=$dbg at=$at $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prio.log)"
done; done; done
