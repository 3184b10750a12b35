set -o pipefail
mkdir -p gpurun_out/wpe
for r in 1 2; do
  for spec in "cur:5:serial" "wpe4:5:serial" "wpe4:5:0.5" "wpe4:5:0.7" "cur:2:d" "wpe4:2:d" "cur:4:d" "wpe4:4:d"; do
    v=${spec%%:*}; rest=${spec#*:}; c=${rest%%:*}; p=${rest#*:}
    e="X=0"; [ $v != cur ] && e="ANA_NATIVE_LIB=ab/${v}_C.so"
    case $p in 0.*) e="$e ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$p";; esac
    env $e timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/wpe/c${c}_${v}_${p}_$r.log 2>&1 || exit 1
    echo "config $c $v prepass $p round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wpe/c${c}_${v}_${p}_$r.log)"
  done
done
