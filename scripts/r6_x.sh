set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
for r in 1 2; do
  for b in 256 320 384; do
    ANA_RATE_BLOCKS=$b ANA_PREPASS_AT=0.55 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/c2_b${b}_$r.log 2>&1 || exit 1
  done
  for t in 0 1; do
    ANA_RATE_TIGHT=$t timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_tight${t}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300 > $O/c5_emu8_head.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config 3 --steps 6 --warmup 2 --force-merge --merges-per-step 16 --emulate-allreduce 8:300 > $O/c3_emu8_head.log 2>&1 || exit 1
python3 - <<'PY'
import glob, re, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6x/*.log")):
    t = open(f).read()
    m = re.search(r'"ms_per_step": ([0-9.]+)', t)
    key = re.sub(r"_\d\.log$", "", f.split("/")[-1])
    rows[key].append(float(m.group(1)) if m else None)
for k, v in sorted(rows.items()):
    print("%-22s %s" % (k, " ".join("%.3f" % x for x in v)))
PY
