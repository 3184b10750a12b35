cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in 0 1 0 1; do echo "== serial=$v"; ANA_PREPASS_SERIAL=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || exit $?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log; done
timeout -k 10 300 python scripts/tune_rate.py --rounds 3 --blocks 512 > gpurun_out/tune.log 2>&1; tail -4 gpurun_out/tune.log
