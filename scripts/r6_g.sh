set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6g2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
C3="python3 bench.py --config 3 --steps 6 --warmup 2 --force-merge"
for r in 1 2; do
  b c3_emu8_auto_$r $C3 --merges-per-step 16 --emulate-allreduce 8:300
  b c3_emu8_at0.5_$r ANA_PREPASS_AT=0.5 $C3 --merges-per-step 16 --emulate-allreduce 8:300
  b c3_emu8_at0.9_$r ANA_PREPASS_AT=0.9 $C3 --merges-per-step 16 --emulate-allreduce 8:300
  b c3_emu8_serial_$r ANA_PREPASS_SERIAL=1 $C3 --merges-per-step 16 --emulate-allreduce 8:300
  b c3_emu8_b512_$r ANA_RATE_BLOCKS=512 $C3 --merges-per-step 16 --emulate-allreduce 8:300
  b c3_emu8_c64_$r ANA_RATE_CHUNK=64 $C3 --merges-per-step 16 --emulate-allreduce 8:300
done
b c3_emu2 $C3 --merges-per-step 2 --emulate-allreduce 2:300
b c3_emu4 $C3 --merges-per-step 8 --emulate-allreduce 4:300
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"prepass_placement": "[^"]*"' $f | tail -1)"; done | sort
