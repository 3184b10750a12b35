set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6t2; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for nb in 2:300 4:300 8:300 8:150 8:600; do
  n=${nb%%:*}
  b e${n}_${nb#*:} python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step $n --emulate-allreduce $nb
done
for n in 2 4 8; do
  b c5e$n python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce $n:300
done
b k8plain python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8
b c2 python3 bench.py --steps 20 --warmup 3
b c5 python3 bench.py --config 5 --steps 10 --warmup 2
b c4 python3 bench.py --config 4 --steps 10 --warmup 2
b worker env DATABASE_URI=columnar:// ENGINE=native BATCHSIZE=500 IDLE_TIMEOUT=0.01 python3 worker.py --synthetic 200000
tail -3 $O/worker.log
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
