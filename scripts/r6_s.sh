set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
B="python3 bench.py --steps 20 --warmup 3"
for r in 1 2; do
  for b in 256 512 768 1024; do
    ANA_RATE_BLOCKS=$b timeout -k 10 300 $B > $O/c2_b${b}_$r.log 2>&1 || exit 1
  done
  ANA_RATE_TIGHT=1 timeout -k 10 300 $B > $O/c2_tight_$r.log 2>&1 || exit 1
  ANA_TELE_TAIL_AT=0.4 timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4_at0.4_$r.log 2>&1 || exit 1
  ANA_TELE_TAIL_AT=0.6 timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4_at0.6_$r.log 2>&1 || exit 1
  timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4_at0.5_$r.log 2>&1 || exit 1
  for at in 0.6 0.85; do
    ANA_PREPASS_AT=$at timeout -k 10 300 $B > $O/c2_at${at}_$r.log 2>&1 || exit 1
  done
  timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_serial_$r.log 2>&1 || exit 1
  ANA_PREPASS_SERIAL=0 timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_tail0.7_$r.log 2>&1 || exit 1
  ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=0.5 timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_tail0.5_$r.log 2>&1 || exit 1
  for b in 512 1024; do
    ANA_RATE_BLOCKS=$b timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 2 > $O/c5_b${b}_$r.log 2>&1 || exit 1
  done
done
for f in $O/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"prepass": "[^"]*"' $f) $(grep -o '"executor_workgroups": [0-9]*' $f)"; done
