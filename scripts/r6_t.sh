set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
B="python3 bench.py --steps 20 --warmup 3"
for r in 1 2 3; do
  for at in 0.45 0.55 0.65 0.75; do
    ANA_PREPASS_AT=$at timeout -k 10 300 $B > $O/c2_at${at}_$r.log 2>&1 || exit 1
  done
  ANA_RATE_BLOCKS=512 ANA_PREPASS_AT=0.3 timeout -k 10 300 $B > $O/c2_b512_at0.3_$r.log 2>&1 || exit 1
  for at in 0.3 0.4 0.5; do
    ANA_TELE_TAIL_AT=$at timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4_at${at}_$r.log 2>&1 || exit 1
  done
  timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_serial_$r.log 2>&1 || exit 1
  ANA_PREPASS_SERIAL=0 timeout -k 10 300 python3 bench.py --config 3 --steps 8 --warmup 2 > $O/c3_tail0.7_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import glob, re, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6t/*.log")):
    m = re.search(r'"ms_per_step": ([0-9.]+)', open(f).read())
    key = re.sub(r"_\d\.log$", "", f.split("/")[-1])
    rows[key].append(float(m.group(1)) if m else None)
for k, v in sorted(rows.items()):
    print("%-22s %s" % (k, " ".join("%.3f" % x for x in v)))
PY
