set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6f3; mkdir -p $O
timeout -k 10 600 python3 scripts/merges_vs_ranks.py --pairs 8x5,8x6,8x8 > $O/sim.log 2>&1 || { tail -5 $O/sim.log; exit 1; }
cat $O/sim.log | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['ranks'], d['merges_per_step'], {k:d[k] for k in d if 'spearman' in k or 'records_dmu_median' in k or 'clamps' in k})"
for k in 5 6; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step $k --emulate-allreduce 8:300 > $O/e8_k$k.log 2>&1 || exit 1
  echo "e8_k$k $(grep -o '"ms_per_step": [0-9.]*' $O/e8_k$k.log)"
done
ANA_DIST_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 8 --steps 2 --warmup 1 --merges-per-step 6 > $O/gloo8_k6.log 2>&1 || { tail -5 $O/gloo8_k6.log; exit 1; }
grep '^{"metric' $O/gloo8_k6.log | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); a=d['accuracy']; print('gloo8 k6', {k:a[k] for k in a if 'spearman' in k or 'records_dmu' in k or 'clamp' in k})"
