set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6i3; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  b s2_l1_$r python3 bench.py --skew 2 --steps 4 --warmup 1
  b s2_l0_$r ANA_RATE_LOCAL=0 python3 bench.py --skew 2 --steps 4 --warmup 1
  b s2_idle1_$r ANA_RATE_IDLE=1 python3 bench.py --skew 2 --steps 4 --warmup 1
  b s2_b192_$r ANA_RATE_BLOCKS=192 python3 bench.py --skew 2 --steps 4 --warmup 1
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
