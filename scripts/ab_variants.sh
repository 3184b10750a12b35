#!/bin/bash
# In-call A/B of experiment builds (ab/<name>_C.so) against the production library:
#   bash scripts/ab_variants.sh NAME...
# interleaved 10M-window executor times (tune_rate.py random), serial-chain hop, and the
# config 2 bench step per library.
set -o pipefail
mkdir -p gpurun_out/abv
for i in 1 2 3; do
  for v in cur "$@"; do
    lib=""; [ $v != cur ] && lib="ANA_NATIVE_LIB=ab/${v}_C.so"
    env $lib timeout -k 10 200 python scripts/tune_rate.py --pattern random --rounds 2 > gpurun_out/abv/r_${v}_$i.log 2>&1 || { echo "!! $v $i"; tail -20 gpurun_out/abv/r_${v}_$i.log; exit 1; }
    env $lib timeout -k 10 100 python scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 > gpurun_out/abv/s_${v}_$i.log 2>&1 || { echo "!! serial $v $i"; exit 1; }
    env $lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/abv/b_${v}_$i.log 2>&1 || { echo "!! bench $v $i"; tail -5 gpurun_out/abv/b_${v}_$i.log; exit 1; }
    echo "$v $i window $(grep '^round 1' gpurun_out/abv/r_${v}_$i.log | grep -o 'rate *[0-9.]* ms') | hop $(grep '^round 1' gpurun_out/abv/s_${v}_$i.log | grep -o '[0-9.]* us per hop') | step $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv/b_${v}_$i.log)"
  done
done
