set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6w2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
E8="python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300"
for r in 1 2; do
  b e8_scan_$r $E8
  b e8_split_next_$r ANA_DP_SPLIT=1 $E8
  b e8_split_tail_$r ANA_DP_SPLIT=1 ANA_DP_DEFER=tail $E8
  b e8_split_now_$r ANA_DP_SPLIT=1 ANA_DP_DEFER=now $E8
  b e8_at0.8_$r ANA_PREPASS_AT=0.8 $E8
  b e8_at0.95_$r ANA_PREPASS_AT=0.95 $E8
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
