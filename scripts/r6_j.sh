set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6j; mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/emu8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --force-merge --merges-per-step 8 --emulate-allreduce 8:300 > $GRAFT_REPO_ROOT/$O/emu8.log 2>&1) || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/c5.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/emu8 -name '*kernel_trace.csv') 80 > $O/emu8_summary.txt
python3 scripts/prof_summary.py $(find $O/c5 -name '*kernel_trace.csv') 40 > $O/c5_summary.txt
head -20 $O/emu8_summary.txt
