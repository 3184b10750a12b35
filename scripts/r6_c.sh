set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6c; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  for c in 64 32 16; do
    b c2_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --steps 20 --warmup 3
  done
  b c2_c32_b512_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=512 python3 bench.py --steps 20 --warmup 3
  for c in 64 32; do
    b c5_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --config 5 --steps 10 --warmup 2
    b c3_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --config 3 --steps 8 --warmup 2
  done
done
for c in 64 32 16; do
  b s3_c$c ANA_RATE_CHUNK=$c python3 bench.py --skew 3 --steps 2 --warmup 1
  b ser_c$c ANA_RATE_CHUNK=$c python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*\|[0-9.]* us per hop' $f | tail -1)"; done | sort
