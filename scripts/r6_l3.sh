set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6l3; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  for p in 2 3 4; do b c5_p${p}_$r ANA_LINK_PARTS=$p python3 bench.py --config 5 --steps 10 --warmup 2; done
  for p in 2 3; do b c3_p${p}_$r ANA_LINK_PARTS=$p python3 bench.py --config 3 --steps 8 --warmup 2; done
  b c2_p2_$r ANA_LINK_PARTS=2 python3 bench.py --steps 20 --warmup 3
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
