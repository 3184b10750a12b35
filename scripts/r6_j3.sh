set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6j3; mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/c3.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/c3 -name '*kernel_trace.csv') 30 > $O/c3_summary.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rr -o run --output-format csv -- python3 -m analyzer_amd.runtime.rerate --matches 3.2e8 --players 1e7 --window 1.6e7 --checkpoint-dir /tmp/ckprof --checkpoint-every 8 > $GRAFT_REPO_ROOT/$O/rr.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/rr -name '*kernel_trace.csv') 40 > $O/rr_summary.txt
grep -o '"ms_per_step": [0-9.]*' $O/c3.log; head -4 $O/c3_summary.txt; head -4 $O/rr_summary.txt
