set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6k3; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  b c3_d1_$r python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_d2_$r ANA_PREPASS_DEPTH=2 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_d2_at0.9_$r ANA_PREPASS_DEPTH=2 ANA_PREPASS_AT=0.9 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_d2_at0.2_$r ANA_PREPASS_DEPTH=2 ANA_PREPASS_AT=0.2 python3 bench.py --config 3 --steps 8 --warmup 2
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
