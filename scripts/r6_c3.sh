set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r6c3; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_rerate_gpu.py tests/test_rerate.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
RR="python3 -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7 --checkpoint-every 8"
rm -rf /tmp/ckfull /tmp/ckkill
timeout -k 10 300 $RR --checkpoint-dir /tmp/ckfull --digests > $O/full.log 2>&1 || exit 1
timeout -k 10 300 $RR --checkpoint-dir /tmp/ckkill --fault-kill-after 20 > $O/kill.log 2>&1; rc=$?
if [ $rc -ne 17 ]; then echo "expected exit 17, got $rc"; tail -5 $O/kill.log; exit 1; fi
timeout -k 10 300 $RR --checkpoint-dir /tmp/ckkill --digests > $O/resume.log 2>&1 || exit 1
python3 - <<'PY'
import json
full = json.loads(open("gpurun_out/r6c3/full.log").read().strip().splitlines()[-1])
res = json.loads(open("gpurun_out/r6c3/resume.log").read().strip().splitlines()[-1])
same = all(full["window_digests"][g] == d for g, d in res["window_digests"].items())
print("resumed from window", int(res["resumed_from_window"]), "| roster bit-identical:", full["roster_sha256"] == res["roster_sha256"],
      "| re-rated windows' records identical:", same, "| seconds full", round(full["seconds"], 3), "| resumed run", round(res["seconds"], 3))
PY
