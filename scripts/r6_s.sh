set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6s2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "handoff or chunk_length or grid_and_register or skew or device" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
P=ab/prev_C.so
b c2_verify python3 bench.py --steps 10 --warmup 2 --verify
grep -o '"verify": {[^}]*}' $O/c2_verify.log
for r in 1 2 3; do
  b c2_new_$r python3 bench.py --steps 20 --warmup 3
  b c2_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --steps 20 --warmup 3
done
for r in 1 2; do
  b c5_new_$r python3 bench.py --config 5 --steps 10 --warmup 2
  b c5_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --config 5 --steps 10 --warmup 2
  b c3_new_$r python3 bench.py --config 3 --steps 8 --warmup 2
  b c3_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --config 3 --steps 8 --warmup 2
  b c4_new_$r python3 bench.py --config 4 --steps 10 --warmup 2
  b c4_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --config 4 --steps 10 --warmup 2
  b s3_new_$r python3 bench.py --skew 3 --steps 2 --warmup 1
  b s3_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --skew 3 --steps 2 --warmup 1
  b s2_new_$r python3 bench.py --skew 2 --steps 4 --warmup 1
  b s2_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --skew 2 --steps 4 --warmup 1
  b ser_new_$r python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --idle 0
  b ser_prev_$r ANA_NATIVE_LIB=$P python3 scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 --idle 0
  b e8_new_$r python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300
  b e8_prev_$r ANA_NATIVE_LIB=$P python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*\|[0-9.]* us per hop' $f | tail -1)"; done | sort
