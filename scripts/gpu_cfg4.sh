#!/bin/bash
# config 4 (fused telemetry) A/B of executor variants + separate mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in 0 1; do ANA_RATE_VARIANT=$v timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/c4.log 2>&1 || { tail -5 gpurun_out/c4.log; exit 1; }; echo "fused v=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4.log)"; done
timeout -k 10 300 python bench.py --config 4 --telemetry-mode separate --steps 10 --warmup 3 > gpurun_out/c4.log 2>&1 || exit 1; echo "separate $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4.log)"
done
timeout -k 10 300 python bench.py --config 3 --steps 6 --warmup 2 > gpurun_out/c3.log 2>&1 || exit 1; echo "config3 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3.log)"
