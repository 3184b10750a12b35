set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6r2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
L=ab/lh1_C.so
for r in 1 2; do
  b c2_prod_$r python3 bench.py --steps 20 --warmup 3
  b c2_l0_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=0 python3 bench.py --steps 20 --warmup 3
  b c2_l1_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=1 python3 bench.py --steps 20 --warmup 3
  b c3_prod_$r python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_l1_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=1 python3 bench.py --config 3 --steps 8 --warmup 2
  b c5_prod_$r python3 bench.py --config 5 --steps 10 --warmup 2
  b c5_l1_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=1 python3 bench.py --config 5 --steps 10 --warmup 2
  b c4_prod_$r python3 bench.py --config 4 --steps 10 --warmup 2
  b c4_l1_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=1 python3 bench.py --config 4 --steps 10 --warmup 2
  b s2_prod_$r python3 bench.py --skew 2 --steps 4 --warmup 1
  b s2_l1_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=1 python3 bench.py --skew 2 --steps 4 --warmup 1
  b s3_prod_$r python3 bench.py --skew 3 --steps 2 --warmup 1
  b s3_l1_$r ANA_NATIVE_LIB=$L ANA_RATE_LOCAL=1 python3 bench.py --skew 3 --steps 2 --warmup 1
  b ser_prod_$r python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --idle 0
  b ser_l1_$r ANA_NATIVE_LIB=$L python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --idle 0 --local 1
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*\|[0-9.]* us per hop' $f | tail -1)"; done | sort
