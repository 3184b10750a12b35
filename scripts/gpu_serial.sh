#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 0 1 0 1; do
  echo -n "serial=$v "; ANA_PREPASS_SERIAL=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])" || exit 1
done
