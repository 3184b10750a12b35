set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6a3; mkdir -p $O
RR="python3 -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7"
for r in 1 2; do
  rm -rf /tmp/cka; timeout -k 10 300 $RR --checkpoint-dir /tmp/cka --checkpoint-every 8 > $O/ck8_$r.log 2>&1 || exit 1
  rm -rf /tmp/cka; ANA_CKPT_FSYNC=0 timeout -k 10 300 $RR --checkpoint-dir /tmp/cka --checkpoint-every 8 > $O/ck8_nofsync_$r.log 2>&1 || exit 1
  rm -rf /tmp/cka; ANA_CKPT_DIRECT=0 timeout -k 10 300 $RR --checkpoint-dir /tmp/cka --checkpoint-every 8 > $O/ck8_buffered_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r6a3/*.log")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["seconds"],3), {k:round(v,4) for k,v in d.items() if k.startswith("checkpoint_")})
PY
