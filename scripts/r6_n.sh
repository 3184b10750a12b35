set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6n; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
C5="python3 bench.py --config 5 --steps 10 --warmup 2"
C3="python3 bench.py --config 3 --steps 8 --warmup 2"
for r in 1 2; do
  b c5_def_$r $C5
  b c5_at0_$r ANA_PREPASS_AT=0.01 $C5
  b c5_at0.2_$r ANA_PREPASS_AT=0.2 $C5
  b c5_nt0_$r ANA_SORT_NT=0 $C5
  b c5_nt1_$r ANA_SORT_NT=1 $C5
  b c5_cus64_$r ANA_PREPASS_CUS=64 $C5
  b c5_cus128_$r ANA_PREPASS_CUS=128 $C5
  b c3_def_$r $C3
  b c3_nt0_$r ANA_SORT_NT=0 $C3
  b c3_nt1_$r ANA_SORT_NT=1 $C3
  b c3_cus64_$r ANA_PREPASS_CUS=64 $C3
  b c3_at0.4_$r ANA_PREPASS_AT=0.4 $C3
  b c3_at0.6_$r ANA_PREPASS_AT=0.6 $C3
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
