set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6pmc2; mkdir -p $O
for l in 0 1; do
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM"; do
    name=$(echo $set | cut -d' ' -f1)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $GRAFT_REPO_ROOT/$O/l$l/$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tune_rate.py --skew 3 --matches 2000000 --blocks 256 --idle 0 --local $l --rounds 1 > $GRAFT_REPO_ROOT/$O/l${l}_$name.log 2>&1) || { echo "FAIL l$l $name"; tail -5 $O/l${l}_$name.log; exit 1; }
    python3 scripts/pmc_kernel.py "$O/l$l/$name" rate_dataflow >> $O/l$l.txt
  done
  grep -E "^round" $O/l${l}_SQ_WAVES.log | cut -c1-200
done
paste $O/l0.txt $O/l1.txt
