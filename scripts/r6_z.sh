set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6z; mkdir -p $O
b() { # name env... -- args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2; do
  b c5_d1_$r ANA_PREPASS_DEPTH=1 python3 bench.py --config 5 --steps 10 --warmup 2
  b c5_d2_$r ANA_PREPASS_DEPTH=2 python3 bench.py --config 5 --steps 10 --warmup 2
  b c5_d2_at0.5_$r ANA_PREPASS_DEPTH=2 ANA_PREPASS_AT=0.5 python3 bench.py --config 5 --steps 10 --warmup 2
  b c2_d1_$r ANA_PREPASS_DEPTH=1 python3 bench.py --steps 20 --warmup 3
  b c2_d2_$r ANA_PREPASS_DEPTH=2 python3 bench.py --steps 20 --warmup 3
  b c3_d1_$r ANA_PREPASS_DEPTH=1 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_d2_$r ANA_PREPASS_DEPTH=2 ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=0.5 python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_d2_at0.9_$r ANA_PREPASS_DEPTH=2 ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=0.9 python3 bench.py --config 3 --steps 8 --warmup 2
  b c4_d1_$r ANA_PREPASS_DEPTH=1 python3 bench.py --config 4 --steps 10 --warmup 2
  b c4_d2_$r ANA_PREPASS_DEPTH=2 python3 bench.py --config 4 --steps 10 --warmup 2
done
RR="python3 -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7 --checkpoint-every 8"
for r in 1 2; do
  for d in 1 2; do
    rm -rf /tmp/ckab
    b rr_d${d}_$r ANA_PREPASS_DEPTH=$d $RR --checkpoint-dir /tmp/ckab
  done
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*\|"seconds": [0-9.]*' $f | tail -1)"; done | sort
