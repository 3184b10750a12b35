set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6x2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2 3; do
  b k4_off_$r python3 bench.py --team-size 4 --steps 8 --warmup 2
  b k4_on_$r ANA_NATIVE_LIB=ab/k4_C.so python3 bench.py --team-size 4 --steps 8 --warmup 2
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
