set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6f2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chunk_length or grid_and_register or five or 5v5 or K5 or team" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
b c3_verify python3 bench.py --config 3 --steps 4 --warmup 2 --verify
grep -o '"verify": {[^}]*}' $O/c3_verify.log
for r in 1 2 3; do
  b c3_$r python3 bench.py --config 3 --steps 8 --warmup 2
  b k4_$r python3 bench.py --team-size 4 --steps 8 --warmup 2
  b c2_$r python3 bench.py --steps 20 --warmup 3
done
for r in 1 2; do
  b c3_emu8_auto_$r python3 bench.py --config 3 --steps 4 --warmup 2 --force-merge --emulate-allreduce 8:300
  b c3_emu8_serial_$r ANA_PREPASS_SERIAL=1 python3 bench.py --config 3 --steps 4 --warmup 2 --force-merge --emulate-allreduce 8:300
  b c3_emu8_b512_$r ANA_RATE_BLOCKS=512 python3 bench.py --config 3 --steps 4 --warmup 2 --force-merge --emulate-allreduce 8:300
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1) $(grep -o '"prepass": "[^"]*"\|"prepass_placement": "[^"]*"' $f | tail -1)"; done | sort
