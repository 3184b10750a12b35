set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6w; mkdir -p $O
for r in 1 2; do
  C5="python3 bench.py --config 5 --steps 6 --warmup 2 --force-merge --merges-per-step 1 --emulate-allreduce 8:300"
  timeout -k 10 300 $C5 > $O/c5_tail0.9_$r.log 2>&1 || exit 1
  ANA_PREPASS_AT=0.1 timeout -k 10 300 $C5 > $O/c5_tail0.1_$r.log 2>&1 || exit 1
  ANA_PREPASS_AT=0.5 timeout -k 10 300 $C5 > $O/c5_tail0.5_$r.log 2>&1 || exit 1
  ANA_DP_SERIAL_AR_US=40 timeout -k 10 300 $C5 > $O/c5_serial_$r.log 2>&1 || exit 1
  C3="python3 bench.py --config 3 --steps 6 --warmup 2 --force-merge --merges-per-step 16 --emulate-allreduce 8:300"
  timeout -k 10 300 $C3 > $O/c3_tail0.7_$r.log 2>&1 || exit 1
  ANA_DP_SERIAL_AR_US=40 timeout -k 10 300 $C3 > $O/c3_serial_$r.log 2>&1 || exit 1
  ANA_PREPASS_AT=0.9 timeout -k 10 300 $C3 > $O/c3_tail0.9_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import glob, re, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6w/*.log")):
    m = re.search(r'"ms_per_step": ([0-9.]+)', open(f).read())
    key = re.sub(r"_\d\.log$", "", f.split("/")[-1])
    rows[key].append(float(m.group(1)) if m else None)
for k, v in sorted(rows.items()):
    print("%-22s %s" % (k, " ".join("%.3f" % x for x in v)))
PY
