#!/bin/bash
# Executor staging loads: records / links through non-temporal loads (ANA_RATE_DEBUG 16 / 32),
# same-process A/B of the executor alone, then bench.py config 2 with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_rate.py --rounds 4 --blocks 512 --debug 0,16,48 > gpurun_out/ntstage.log 2>&1 || { tail -5 gpurun_out/ntstage.log; exit 1; }
grep round gpurun_out/ntstage.log | tail -6
for d in 0 16 48 0 16 48; do
  ANA_RATE_DEBUG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 3 --check > gpurun_out/ntbench.log 2>&1 || { tail -5 gpurun_out/ntbench.log; exit 1; }
  echo "debug=$d $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ntbench.log)"
done
