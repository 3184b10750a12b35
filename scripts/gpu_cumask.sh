#!/bin/bash
# Bench with the schedule side stream confined to N CUs (ANA_PREPASS_CUS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in ${CUS:-0 32 64 128 0}; do
  echo -n "cus=$n "; ANA_PREPASS_CUS=$n timeout -k 10 300 python bench.py --steps 10 --warmup 3 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])" || exit 1
done
