#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ANA_RATE_TIGHT=1 timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -1 || exit 1
run() { echo "== $*"; timeout -k 10 300 python scripts/tune_rate.py --rounds 3 "$@" > gpurun_out/micro.log 2>&1; rc=$?; tail -1 gpurun_out/micro.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d['by_blocks'].items(): print(k, 'sched %.2f rate %.2f (median %.2f)' % (v['schedule_ms_min'], v['rate_ms_min'], v['rate_ms_median']))"; [ $rc -eq 0 ] || exit $rc; }
run --pattern random --players 1000000 --matches 10000000 --blocks 512 --tight 0,1
run --pattern random --players 1000000 --matches 12500000 --team-size 5 --blocks 512 --tight 0,1
run --pattern disjoint --players 6000000 --matches 1000000 --blocks 1024 --tight 0,1
