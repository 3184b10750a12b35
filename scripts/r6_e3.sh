set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6e3; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
C5="python3 bench.py --config 5 --steps 10 --warmup 2"
for r in 1 2; do
  b c5_b512_$r $C5
  b c5_b384_$r ANA_RATE_BLOCKS=384 $C5
  b c5_b256_$r ANA_RATE_BLOCKS=256 $C5
  b c5_b640_$r ANA_RATE_BLOCKS=640 $C5
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"prepass": "[^"]*"' $f | tail -1)"; done | sort
