#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $ROOT/gpurun_out/pmc/counters.txt 2>&1 || true
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INST_LEVEL_VMEM SQ_INSTS_FLAT"; do
  name=$(echo $set | cut -d' ' -f1)
  echo "== pmc $set"
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --stats -d $ROOT/gpurun_out/pmc/$name -o run --output-format csv -- python3 $ROOT/scripts/tune_rate.py --rounds 1 ${TUNE_ARGS:---pattern disjoint --players 6000000 --matches 1000000 --blocks 1024} > $ROOT/gpurun_out/pmc/$name.log 2>&1; rc=$?
  tail -1 $ROOT/gpurun_out/pmc/$name.log | cut -c1-200
  [ $rc -eq 0 ] || echo "rc=$rc (continuing only if not a crash)"
  if [ $rc -gt 1 ] && [ $rc -ne 124 ]; then exit $rc; fi
done
