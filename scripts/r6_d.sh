set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6d2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  for c in 32 16 8; do
    b c3_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --config 3 --steps 8 --warmup 2
  done
  b c3_c16_b1024_$r ANA_RATE_CHUNK=16 ANA_RATE_BLOCKS=1024 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c32_b1024_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=1024 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c32_b256_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=256 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c32_tail_$r ANA_RATE_CHUNK=32 ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=0.7 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c32_tight_$r ANA_RATE_CHUNK=32 ANA_RATE_TIGHT=1 python3 bench.py --config 3 --steps 8 --warmup 2
  for c in 64 32 16; do
    b k4_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --team-size 4 --steps 8 --warmup 2
  done
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*\|[0-9.]* us per hop' $f | tail -1)"; done | sort
