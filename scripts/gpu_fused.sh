#!/bin/bash
# config 4 fused-telemetry policy A/B (tail-only vs any idle wave) + separate reference
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tele
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused" > gpurun_out/tele/pytest_fused.log 2>&1 || { tail -30 gpurun_out/tele/pytest_fused.log; exit 1; }
tail -1 gpurun_out/tele/pytest_fused.log
for rep in 1 2; do
for tail in 1 0; do
  ANA_TELE_FUSED_TAIL=$tail timeout -k 10 300 python bench.py --config 4 --telemetry-mode fused --steps 10 --warmup 3 > gpurun_out/tele/c4f.log 2>&1 || { tail -20 gpurun_out/tele/c4f.log; exit 1; }
  echo "fused tail=$tail $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tele/c4f.log)"
done
timeout -k 10 300 python bench.py --config 4 --telemetry-mode separate --steps 10 --warmup 3 > gpurun_out/tele/c4s.log 2>&1 || exit 1
echo "separate $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tele/c4s.log)"
done
