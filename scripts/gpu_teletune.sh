#!/bin/bash
# K8 telemetry kernel: variant timing + one PMC pass per counter set on the default kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out/tele
timeout -k 10 300 python scripts/tune_tele.py --variants "${VARIANTS:-impl0,dbg1,dbg2}" > gpurun_out/tele/tune.log 2>&1 || { tail -20 gpurun_out/tele/tune.log; exit 1; }
grep -v '^{' gpurun_out/tele/tune.log | tail -9
[ -n "$NOPMC" ] && exit 0
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" "SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/tele/p$i -o run --output-format csv -- python3 $ROOT/scripts/tune_tele.py --variants ${PMCVAR:-impl0} --rounds 1 --iters 1 > $ROOT/gpurun_out/tele/p$i.log 2>&1; rc=$?
  echo "set $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
