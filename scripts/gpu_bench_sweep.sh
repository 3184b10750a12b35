#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${BLOCKS:-256 512}; do
  echo "== bench blocks=$b"; ANA_RATE_BLOCKS=$b timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$b.log 2>&1; rc=$?
  tail -1 gpurun_out/bench_$b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])"; [ $rc -eq 0 ] || exit $rc
done
