#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -1 || exit 1
timeout -k 10 300 python scripts/tune_rate.py --rounds 3 --blocks 512 --packed 0,1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d['by_blocks'].items(): print(k, 'rate %.2f (median %.2f)' % (v['rate_ms_min'], v['rate_ms_median']))" || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 | python3 -c "import json,sys; print('bench', json.loads(sys.stdin.read())['ms_per_step'])" || exit 1; done
