set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6fin; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.log | head; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_default.log 2>&1 || { tail $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --check --verify > $O/bench_verify.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"verify": {[^}]*}' $O/bench_verify.log | head -3
