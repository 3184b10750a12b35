set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6i; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
E8="python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300"
for r in 1 2; do
  b emu8_c64_$r $E8
  b emu8_c48_$r ANA_RATE_CHUNK=48 $E8
  b emu8_c32_$r ANA_RATE_CHUNK=32 $E8
  b emu8_b384_$r ANA_RATE_BLOCKS=384 $E8
  b emu8_b512_$r ANA_RATE_BLOCKS=512 $E8
  b k8plain_$r python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8
  b plain_$r python3 bench.py --steps 20 --warmup 3
  b s3_b192_$r ANA_RATE_BLOCKS=192 python3 bench.py --skew 3 --steps 2 --warmup 1
  b s3_b256_$r python3 bench.py --skew 3 --steps 2 --warmup 1
done
for f in $O/*.log; do n=$(basename $f .log); echo "$n $(grep -o '"ms_per_step": [0-9.]*' $f | tail -1)"; done | sort
