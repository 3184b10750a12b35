set -o pipefail
mkdir -p gpurun_out/sortv
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sched or schedule or sort or link" > gpurun_out/sortv/tests.log 2>&1 || { tail -5 gpurun_out/sortv/tests.log; exit 1; }
tail -1 gpurun_out/sortv/tests.log
for r in 1 2; do
  for spec in "prev:5:serial" "new:5:serial" "new:5:0.5" "new:5:0.7" "prev:2:d" "new:2:d" "prev:3:d" "new:3:d"; do
    v=${spec%%:*}; rest=${spec#*:}; c=${rest%%:*}; p=${rest#*:}
    e=""; [ $v = prev ] && e="ANA_NATIVE_LIB=ab/prev_C.so"
    case $p in 0.*) e="$e ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$p";; esac
    env $e timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/sortv/c${c}_${v}_${p}_$r.log 2>&1 || exit 1
    echo "config $c $v prepass $p round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sortv/c${c}_${v}_${p}_$r.log)"
  done
done
