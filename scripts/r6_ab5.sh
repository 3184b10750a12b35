set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
for r in 1 2; do
  for v in reg reg2 lds4 lds2; do
    ANA_NATIVE_LIB=ab/${v}_C.so timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_${v}_$r.log 2>&1 || exit 1
    ANA_NATIVE_LIB=ab/${v}_C.so ANA_PREPASS_SERIAL=1 timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_${v}_serial_$r.log 2>&1 || exit 1
  done
done
for f in $O/c3_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"prepass": "[^"]*"' $f)"; done
ANA_NATIVE_LIB=ab/lds4_C.so timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "5 and (host or bit or engine)" > $O/t5_lds4.log 2>&1; tail -1 $O/t5_lds4.log
ANA_NATIVE_LIB=ab/lds2_C.so timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "5 and (host or bit or engine)" > $O/t5_lds2.log 2>&1; tail -1 $O/t5_lds2.log
echo rc=$?
