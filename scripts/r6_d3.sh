set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6d3; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  b c3_def_$r python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_t0c32_$r ANA_RATE_TIGHT=0 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_t0c64_$r ANA_RATE_TIGHT=0 ANA_RATE_CHUNK=64 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_t0c16_$r ANA_RATE_TIGHT=0 ANA_RATE_CHUNK=16 python3 bench.py --config 3 --steps 8 --warmup 2
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
