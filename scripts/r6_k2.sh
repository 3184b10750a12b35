set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6k2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rccl" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
E8="python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300"
for r in 1 2; do
  b e8_b1_$r ANA_DP_CORR_BUCKETS=0 $E8
  b e8_b16mb_$r $E8
  b e8_b8mb_$r ANA_MERGE_BUCKET_MB=8 $E8
  b e8_b16mb_nowarm_$r ANA_ROSTER_WARM=0 $E8
  b e8_b1_nowarm_$r ANA_DP_CORR_BUCKETS=0 ANA_ROSTER_WARM=0 $E8
  b e4_b1_$r ANA_DP_CORR_BUCKETS=0 python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 4 --emulate-allreduce 4:300
  b e4_b16mb_$r python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 4 --emulate-allreduce 4:300
  b c5e8_b1_$r ANA_DP_CORR_BUCKETS=0 python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300
  b c5e8_b16mb_$r python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300
  b c5e8_b64mb_$r ANA_MERGE_BUCKET_MB=64 python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
