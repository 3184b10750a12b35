#!/bin/bash
# K8 one-hot MFMA telemetry: GPU numerics tests, impl A/B timing, config 4 bench (fused + separate)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tele
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "telemetry" > gpurun_out/tele/pytest.log 2>&1 || { tail -40 gpurun_out/tele/pytest.log; exit 1; }
tail -2 gpurun_out/tele/pytest.log
timeout -k 10 300 python scripts/tune_tele.py --variants "${VARIANTS:-impl1,impl0}" > gpurun_out/tele/tune_mfma.log 2>&1 || { tail -20 gpurun_out/tele/tune_mfma.log; exit 1; }
grep -v '^{' gpurun_out/tele/tune_mfma.log | tail -6
for mode in ${MODES:-overlap fused separate}; do
  timeout -k 10 300 python bench.py --config 4 --telemetry-mode $mode --steps 10 --warmup 3 > gpurun_out/tele/c4_$mode.log 2>&1 || { tail -20 gpurun_out/tele/c4_$mode.log; exit 1; }
  echo "config4 $mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tele/c4_$mode.log)"
done
