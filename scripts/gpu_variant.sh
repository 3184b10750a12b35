#!/bin/bash
# Same-process A/B of executor variants (ANA_RATE_VARIANT), random 10M/1M stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_rate.py --rounds ${ROUNDS:-4} --blocks 512 --variant ${VARIANTS:-0,1} ${TUNE_ARGS} > gpurun_out/variant.log 2>&1; rc=$?
grep round gpurun_out/variant.log | tail -8; tail -1 gpurun_out/variant.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d['by_blocks'].items(): print(k, 'sched %.3f rate min %.3f median %.3f' % (v['schedule_ms_min'], v['rate_ms_min'], v['rate_ms_median']))"
exit $rc
