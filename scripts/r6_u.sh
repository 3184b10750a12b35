set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6u; mkdir -p $O
E8="python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce 8:300"
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/c2_head_$r.log 2>&1 || exit 1
  for at in 0.1 0.2 0.3; do
    ANA_TELE_TAIL_AT=$at timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 2 > $O/c4_at${at}_$r.log 2>&1 || exit 1
  done
  for at in 0.0 0.1 0.3; do
    ANA_PREPASS_AT=$at timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 2 > $O/c5_at${at}_$r.log 2>&1 || exit 1
  done
  timeout -k 10 300 $E8 > $O/emu8_serial_$r.log 2>&1 || exit 1
  for at in 0.5 0.9; do
    ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$at timeout -k 10 300 $E8 > $O/emu8_tail${at}_$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import glob, re, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6u/*.log")):
    m = re.search(r'"ms_per_step": ([0-9.]+)', open(f).read())
    key = re.sub(r"_\d\.log$", "", f.split("/")[-1])
    rows[key].append(float(m.group(1)) if m else None)
for k, v in sorted(rows.items()):
    print("%-22s %s" % (k, " ".join("%.3f" % x for x in v)))
PY
