#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 300 python scripts/tune_rate.py --rounds 3 "$@" > gpurun_out/micro.log 2>&1; rc=$?; tail -1 gpurun_out/micro.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d['by_blocks'].items(): print(k, 'sched %.2f rate %.2f (median %.2f)' % (v['schedule_ms_min'], v['rate_ms_min'], v['rate_ms_median']))"; cat gpurun_out/micro.log >> gpurun_out/micro_all.log; [ $rc -eq 0 ] || exit $rc; }
run --pattern random --players 1000000 --matches 10000000 --blocks 512 --spec ${SPEC:-0,1,2,4,8}
run --pattern serial --players 1000 --matches 20000 --blocks 512 --spec ${SPEC:-0,1,2,4,8}
