set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6y2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "handoff or chunk_length" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
for r in 1 2; do timeout -k 10 300 python3 bench.py --team-size 4 --steps 8 --warmup 2 > $O/k4_$r.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' $O/k4_$r.log; done
