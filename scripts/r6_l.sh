set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6l; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  for mb in 0 16 64; do
    b e2_mb${mb}_$r ANA_MERGE_BUCKET_MB=$mb python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 2 --emulate-allreduce 2:300
    b c5e2_mb${mb}_$r ANA_MERGE_BUCKET_MB=$mb python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 2:300
  done
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
