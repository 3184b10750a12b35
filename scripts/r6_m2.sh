set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6m2; mkdir -p $O
timeout -k 10 300 python3 scripts/tune_rate.py --blocks 256 --idle 0 --diag 0,1 --rounds 2 > $O/c2_diag.log 2>&1 || { tail $O/c2_diag.log; exit 1; }
ANA_RATE_CHUNK=32 timeout -k 10 300 python3 scripts/tune_rate.py --team-size 5 --matches 12500000 --blocks 256 --idle 0 --diag 0,1 --rounds 2 > $O/c3_diag.log 2>&1 || { tail $O/c3_diag.log; exit 1; }
grep -E "rate|iter|wait|issue" $O/c2_diag.log | tail -8
grep -E "rate|iter|wait|issue" $O/c3_diag.log | tail -8
