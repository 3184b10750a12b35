set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6e; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  b c3_c64_b256_$r ANA_RATE_CHUNK=64 ANA_RATE_BLOCKS=256 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c64_b128_$r ANA_RATE_CHUNK=64 ANA_RATE_BLOCKS=128 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c32_b192_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=192 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_c32_b320_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=320 python3 bench.py --config 3 --steps 8 --warmup 2
  for at in 0.3 0.5 0.7 0.85; do
    b c3_c32_b256_at${at}_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=256 ANA_PREPASS_AT=$at python3 bench.py --config 3 --steps 8 --warmup 2
  done
  b c3_c32_b256_serial_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=256 ANA_PREPASS_SERIAL=1 python3 bench.py --config 3 --steps 8 --warmup 2
  b k4_c32_b256_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=256 python3 bench.py --team-size 4 --steps 8 --warmup 2
  b k4_c32_b512_$r ANA_RATE_CHUNK=32 ANA_RATE_BLOCKS=512 python3 bench.py --team-size 4 --steps 8 --warmup 2
  b k4_c64_b256_$r ANA_RATE_CHUNK=64 ANA_RATE_BLOCKS=256 python3 bench.py --team-size 4 --steps 8 --warmup 2
  b c2_c64_b128_$r ANA_RATE_CHUNK=64 ANA_RATE_BLOCKS=192 python3 bench.py --steps 20 --warmup 3
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"prepass": "[^"]*"' $f | tail -1)"; done | sort
