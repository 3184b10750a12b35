#!/bin/bash
# Software-pipelined executor (ANA_RATE_VARIANT=5): bit-identity test, same-process A/B
# against the production executor, then bench.py config 2 / 3 with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== test"
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k pipelined -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/pipe_test.log 2>&1; rc=$?
tail -3 gpurun_out/pipe_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B 0,5"
VARIANTS=0,5 bash scripts/gpu_variant.sh || exit $?
for v in 0 5; do
  for c in 2 3; do
    echo "== bench config $c variant $v"
    ANA_RATE_VARIANT=$v timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --check \
      > gpurun_out/pipe_bench_c${c}_v${v}.log 2>&1 || exit $?
    tail -1 gpurun_out/pipe_bench_c${c}_v${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f ms/step' % d['ms_per_step'])"
  done
done
