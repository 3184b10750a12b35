set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
B="python3 bench.py --steps 20 --warmup 3"
for r in 1 2; do
  timeout -k 10 300 $B > $O/base_$r.log 2>&1 || exit 1
  for cus in 64 128; do
    for at in 0.5 0.65 0.75; do
      ANA_PREPASS_CUS=$cus ANA_PREPASS_AT=$at timeout -k 10 300 $B > $O/cus${cus}_at${at}_$r.log 2>&1 || exit 1
    done
  done
  for at in 0.65 0.85; do
    ANA_PREPASS_AT=$at timeout -k 10 300 $B > $O/at${at}_$r.log 2>&1 || exit 1
  done
done
for f in $O/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
E5="python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300"
timeout -k 10 300 $E5 > $O/c5_default.log 2>&1 || exit 1
for at in 0.1 0.3 0.6; do
  ANA_DP_SPLIT=1 ANA_DP_DEFER=tail ANA_DP_DEFER_AT=$at timeout -k 10 300 $E5 > $O/c5_split_tail$at.log 2>&1 || exit 1
done
for f in $O/c5*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"correct_records": [0-9.]*' $f) $(grep -o '"allreduce": [0-9.]*' $f)"; done
