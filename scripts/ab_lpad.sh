#!/bin/bash
# A/B: LDS output-row padding (ANA_LROW_PAD=4, ab/lpad4_C.so) vs the production library,
# interleaved in one call; bank-conflict counter of each.
set -o pipefail
mkdir -p gpurun_out/ab
ROOT=$(pwd)
for i in 1 2 3; do
  for v in cur lpad4; do
    lib=""; [ $v = lpad4 ] && lib="ANA_NATIVE_LIB=ab/lpad4_C.so"
    env $lib timeout -k 10 200 python scripts/tune_rate.py --pattern random --rounds 2 > gpurun_out/ab/lp_${v}_$i.log 2>&1 || { echo "!! $v $i"; tail -20 gpurun_out/ab/lp_${v}_$i.log; exit 1; }
    echo "$v $i $(grep '^round 1' gpurun_out/ab/lp_${v}_$i.log | grep -o 'rate *[0-9.]* ms')"
  done
done
for v in cur lpad4; do
  lib=""; [ $v = lpad4 ] && lib="$ROOT/ab/lpad4_C.so"
  (cd /tmp && ANA_NATIVE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --kernel-trace --stats \
      -d "$ROOT/gpurun_out/ab/pmc_$v" -o run --output-format csv -- python3 "$ROOT/scripts/tune_rate.py" --rounds 1 \
      > "$ROOT/gpurun_out/ab/pmc_$v.log" 2>&1) || { echo "!! pmc $v"; exit 1; }
  echo "pmc $v"; python3 scripts/pmc_kernel.py "gpurun_out/ab/pmc_$v" rate_dataflow
done
