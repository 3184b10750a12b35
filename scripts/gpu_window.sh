#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for m in 10000000 5000000 2500000; do
  echo -n "M=$m "; timeout -k 10 300 python scripts/tune_rate.py --rounds 3 --blocks 512 --matches $m | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d['by_blocks'].items(): print('sched %.2f rate %.2f' % (v['schedule_ms_min'], v['rate_ms_min']))" || exit 1
done
