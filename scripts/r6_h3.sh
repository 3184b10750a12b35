set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6h3; mkdir -p $O
b() { local name=$1; shift
  timeout -k 10 400 env "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
}
for r in 1 2 3; do
  for at in 0.45 0.55 0.65; do b c2_at${at}_$r ANA_PREPASS_AT=$at python3 bench.py --steps 20 --warmup 3; done
  for at in 0.1 0.2 0.3; do b c4_at${at}_$r ANA_TELE_TAIL_AT=$at python3 bench.py --config 4 --steps 10 --warmup 2; done
done
python3 - <<'PY'
import glob,re,collections
d=collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6h3/*.log")):
    n=f.split("/")[-1][:-4]; k=n.rsplit("_",1)[0]
    m=re.findall(r'"ms_per_step": ([0-9.]+)', open(f).read())
    d[k].append(float(m[-1]))
for k,v in sorted(d.items()): print("%-14s %s" % (k, " ".join("%.3f" % x for x in v)))
PY
