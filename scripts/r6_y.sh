set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_rerate_gpu.py tests/test_rerate.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
RR="python3 -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7 --checkpoint-every 8"
for r in 1 2; do
  for m in main tail; do
    rm -rf /tmp/ckab
    ANA_RERATE_GEN=$m timeout -k 10 300 $RR --checkpoint-dir /tmp/ckab > $O/rr_${m}_$r.log 2>&1 || exit 1
    echo "rr_${m}_$r $(tail -1 $O/rr_${m}_$r.log | grep -o '"seconds": [0-9.]*')"
  done
done
rm -rf /tmp/ckfull /tmp/ckkill
timeout -k 10 300 $RR --checkpoint-dir /tmp/ckfull --digests > $O/full.log 2>&1 || exit 1
timeout -k 10 300 $RR --checkpoint-dir /tmp/ckkill --fault-kill-after 20 > $O/kill.log 2>&1; rc=$?
if [ $rc -ne 17 ]; then echo "expected exit 17, got $rc"; tail -5 $O/kill.log; exit 1; fi
timeout -k 10 300 $RR --checkpoint-dir /tmp/ckkill --digests > $O/resume.log 2>&1 || exit 1
python3 - <<'PY'
import json
full = json.loads(open("gpurun_out/r6y/full.log").read().strip().splitlines()[-1])
res = json.loads(open("gpurun_out/r6y/resume.log").read().strip().splitlines()[-1])
g0 = int(res["resumed_from_window"])
same = all(full["window_digests"][g] == d for g, d in res["window_digests"].items())
print("resumed from window", g0, "| roster bit-identical:", full["roster_sha256"] == res["roster_sha256"],
      "| re-rated windows' records identical:", same, "| statuses", {k: full[k] for k in ("rated", "afk") if k in full},
      "| seconds full", round(full["seconds"], 3))
PY
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/rr -o run --output-format csv -- python3 -m analyzer_amd.runtime.rerate --matches 3.2e8 --players 1e7 --window 1.6e7 --checkpoint-dir /tmp/ckprof --checkpoint-every 8 > $GRAFT_REPO_ROOT/$O/rrprof.log 2>&1) || exit 1
python3 scripts/prof_summary.py $(find $O/rr -name '*kernel_trace.csv') 60 > $O/rr_summary.txt
head -30 $O/rr_summary.txt
