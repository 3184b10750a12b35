set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6v2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
H=ab/h2_C.so
for r in 1 2; do
  b c2_h1_$r python3 bench.py --steps 20 --warmup 3
  b c2_h2_$r ANA_NATIVE_LIB=$H python3 bench.py --steps 20 --warmup 3
  b c5_h1_$r python3 bench.py --config 5 --steps 10 --warmup 2
  b c5_h2_$r ANA_NATIVE_LIB=$H python3 bench.py --config 5 --steps 10 --warmup 2
  b s3_h1_$r python3 bench.py --skew 3 --steps 2 --warmup 1
  b s3_h2_$r ANA_NATIVE_LIB=$H python3 bench.py --skew 3 --steps 2 --warmup 1
  b ser_h1_$r python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --idle 0
  b ser_h2_$r ANA_NATIVE_LIB=$H python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --idle 0
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*\|[0-9.]* us per hop' $f | tail -1)"; done | sort
