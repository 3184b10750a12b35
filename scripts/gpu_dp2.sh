#!/bin/bash
# 2-rank rehearsal of the DP sweep-merge bench path on one GPU (gloo; production N>1 uses RCCL),
# fp32 and fp16 merge messages, plus the 1-rank reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --matches-per-gpu 2000000 > gpurun_out/dp1.log 2>&1 || { tail -20 gpurun_out/dp1.log; exit 1; }
grep '"metric"' gpurun_out/dp1.log | cut -c1-400
for dt in fp32 fp16; do
  ANA_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --matches-per-gpu 2000000 --comm-dtype $dt --check > gpurun_out/dp2_$dt.log 2>&1 || { tail -20 gpurun_out/dp2_$dt.log; exit 1; }
  grep '"metric"' gpurun_out/dp2_$dt.log | cut -c1-400
done
