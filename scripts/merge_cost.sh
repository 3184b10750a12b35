# DP merge device cost on one GPU: merge kernel micro-benchmark, then bench.py
# at k = 1 and k = 8 windows per step with and without the merge kernels forced on
set -o pipefail
timeout -k 10 200 python scripts/merge_micro.py --players 1e6,1e7 > gpurun_out/merge_micro.log 2>&1 || exit 1
for args in "--merges-per-step 1" "--merges-per-step 8" "--merges-per-step 8 --force-merge" "--merges-per-step 1 --force-merge"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 $args > gpurun_out/bench_k.log 2>&1 || exit 1
  echo "$args $(tail -1 gpurun_out/bench_k.log)" >> gpurun_out/merge_cost.log
done
