#!/bin/bash
# PMC passes (instruction mix, LDS, waits) of telemetry variants: VARS="impl1s63 dbg7s63"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out/telepmc
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-impl1s63 dbg7s63}; do
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/telepmc/$v/p$i -o run --output-format csv -- python3 $ROOT/scripts/tune_tele.py --variants $v --rounds 1 --iters 1 > $ROOT/gpurun_out/telepmc/$v.p$i.log 2>&1; rc=$?
  echo "$v set $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
