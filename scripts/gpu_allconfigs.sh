#!/bin/bash
# Every bench config on one GPU (writes gpurun_out/bench_configs.log).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; : > gpurun_out/bench_configs.log
for args in "--config 2" "--config 3" "--config 4 --telemetry-mode fused" "--config 4 --telemetry-mode separate" "--config 5"; do
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --check $args > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log >> gpurun_out/bench_configs.log
  tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-40s %8.3f ms  %.4g %s' % ('$args', d['ms_per_step'], d['value'], d['unit']))"
done
# 2-rank rehearsal of the DP merge path on one GPU (gloo; production N>1 uses RCCL)
if [ -n "$DP2" ]; then
  ANA_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --matches-per-gpu 2000000 > gpurun_out/b2.log 2>&1 || { tail -20 gpurun_out/b2.log; exit 1; }
  grep '"metric"' gpurun_out/b2.log | cut -c1-300
fi
