set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6v; mkdir -p $O
for r in 1 2; do
  for at in 0.8 0.9 0.95; do
    ANA_PREPASS_AT=$at timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300 > $O/emu8_at${at}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4_head.log 2>&1 || exit 1
for nb in 2:300 4:300 8:150 8:600; do
  n=${nb%%:*}
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step $n --emulate-allreduce $nb > $O/emu${nb/:/_}.log 2>&1 || exit 1
done
for n in 2 4 8; do
  if [ $n = 2 ]; then k=2; elif [ $n = 4 ]; then k=8; else k=16; fi
  timeout -k 10 300 python3 bench.py --config 3 --steps 6 --warmup 2 --force-merge --merges-per-step $k --emulate-allreduce $n:300 > $O/c3_emu$n.log 2>&1 || exit 1
  timeout -k 10 300 python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce $n:300 > $O/c5_emu$n.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_head.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 2 > $O/c5_head.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --skew 2 --steps 6 --warmup 2 > $O/skew2.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --skew 3 --steps 3 --warmup 1 > $O/skew3.log 2>&1 || exit 1
for f in $O/*.log; do echo "$(basename $f .log) $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"prepass_placement": "[^"]*"' $f)"; done
