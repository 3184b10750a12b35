set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6q; mkdir -p $O
D=$(ls analyzer_amd/_C_diag*.so)
ANA_NATIVE_LIB=$D timeout -k 10 300 python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --local 0,1 --diag 0,1 --idle 0 > $O/serial_local.log 2>&1 || { tail $O/serial_local.log; exit 1; }
ANA_NATIVE_LIB=$D timeout -k 10 300 python3 scripts/tune_rate.py --skew 3 --rounds 1 --blocks 256 --local 0,1 --diag 0,1 --idle 0 > $O/skew3_local.log 2>&1 || { tail $O/skew3_local.log; exit 1; }
grep -E "^round" $O/serial_local.log | cut -c1-400
grep -E "^round" $O/skew3_local.log | cut -c1-400
