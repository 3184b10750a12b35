set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6pmc; mkdir -p $O
for c in 32 64; do
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    name=$(echo $set | cut -d' ' -f1)
    (cd /tmp && ANA_RATE_CHUNK=$c timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $GRAFT_REPO_ROOT/$O/c$c/$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tune_rate.py --team-size 5 --matches 12500000 --blocks 256 --idle 0 --rounds 1 > $GRAFT_REPO_ROOT/$O/c${c}_$name.log 2>&1) || { echo "FAIL c$c $name"; tail -5 $O/c${c}_$name.log; exit 1; }
    python3 scripts/pmc_kernel.py "$O/c$c/$name" rate_dataflow >> $O/c$c.txt
  done
done
paste $O/c32.txt $O/c64.txt
