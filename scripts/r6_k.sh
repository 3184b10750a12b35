set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
for n in 2 4 8; do
  s=$([ $n = 8 ] && echo 2 || echo 3)
  ANA_DIST_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus $n --steps $s --warmup 1 > $O/gloo$n.log 2>&1 || exit 1
  grep -h '^{' $O/gloo$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['accuracy']; print('gloo$n', d['config']['mode'], 'spearman', a['spearman_mu_minus_sigma'], 'records median/p99/max', a['records_dmu_median'], a['records_dmu_p99'], a['records_dmu_max'], 'clamps', a['merge_clamp_hits'])"
done
ANA_DIST_BACKEND=gloo timeout -k 10 900 python3 bench.py --config 5 --gpus 8 --steps 1 --warmup 1 > $O/c5_gloo8.log 2>&1 || exit 1
grep -h '^{' $O/c5_gloo8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['accuracy']; print('c5 gloo8 k', d['config']['merges_per_step'], 'spearman', a['spearman_mu_minus_sigma'], 'records median/p99/max', a['records_dmu_median'], a['records_dmu_p99'], a['records_dmu_max'], 'clamps', a['merge_clamp_hits'])"
for n in 1 2 4; do
  for mode in cas racy; do
    rm -f /tmp/rep$n$mode.db*
    cas=$([ $mode = racy ] && echo 0 || echo auto)
    PLAYER_CAS=$cas ENGINE=native DATABASE_URI=sqlite:////tmp/rep$n$mode.db timeout -k 10 600 python3 worker.py --synthetic 40000 --replicas $n > $O/replicas_${mode}_$n.log 2>&1 || exit 1
    grep -h '^{' $O/replicas_${mode}_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('replicas', '$mode', $n, 'matches/s %.0f' % d['matches_per_s'], 'cas_retries', d.get('cas_retries'), 'unsettled', d.get('unsettled'))"
  done
done

bash scripts/gpu.sh rerate > $O/rerate_task.log 2>&1; rc=$?; tail -4 $O/rerate_task.log; cp -r gpurun_out/rerate $O/ 2>/dev/null; exit $rc
