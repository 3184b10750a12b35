set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6u2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  b wk_new_$r python3 scripts/worker_profile.py --synthetic 200000 --cprofile 0 --segments 4
  b wk_prev_$r ANA_NATIVE_LIB=ab/prev_C.so python3 scripts/worker_profile.py --synthetic 200000 --cprofile 0 --segments 4
  b wkp_new_$r python3 scripts/worker_profile.py --synthetic 200000 --cprofile 0 --segments 4 --pipeline true
  b wkp_prev_$r ANA_NATIVE_LIB=ab/prev_C.so python3 scripts/worker_profile.py --synthetic 200000 --cprofile 0 --segments 4 --pipeline true
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"matches_per_s": [0-9.]*\|"segment_matches_per_s_median": [0-9.]*' $f | tr '\n' ' ')"; done | sort
