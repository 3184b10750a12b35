set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6h2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  for c in 24 32 40 48; do b c3_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --config 3 --steps 8 --warmup 2; done
  for c in 40 48 56 64; do b c2_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --steps 20 --warmup 3; done
  b c2_c48_b320_$r ANA_RATE_CHUNK=48 ANA_RATE_BLOCKS=320 python3 bench.py --steps 20 --warmup 3
  for c in 48 64; do b c5_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --config 5 --steps 10 --warmup 2; done
  for c in 40 48 64; do b k4_c${c}_$r ANA_RATE_CHUNK=$c python3 bench.py --team-size 4 --steps 8 --warmup 2; done
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
