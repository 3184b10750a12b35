set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6p; mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/c2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/c2.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/c2 -name '*kernel_trace.csv') 40 > $O/c2_summary.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/c3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/c3.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/c3 -name '*kernel_trace.csv') 30 > $O/c3_summary.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/rr -o run --output-format csv -- python3 -m analyzer_amd.runtime.rerate --matches 1.6e8 --players 1e7 --window 1.6e7 --records digest --checkpoint-dir /tmp/ckprof --checkpoint-every 4 > $GRAFT_REPO_ROOT/$O/rr.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/rr -name '*kernel_trace.csv') 30 > $O/rr_summary.txt
head -24 $O/c2_summary.txt
