set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --check --verify > $O/bench_verify.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"max_abs_dmu[^,]*\|"status_mismatch[^,]*' $O/bench_verify.log | head -5
for r in 1 2; do
  for v in cur h5_1; do
    ANA_NATIVE_LIB=ab/${v}_C.so timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_${v}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300 > $O/emu8.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300 > $O/c5_emu8.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 2 > $O/c5.log 2>&1 || exit 1
for f in $O/c*.log $O/emu8.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
