set -o pipefail
GTEST_K="sweep or packed or record or decode or distributed or rccl or merge" bash scripts/gpu.sh gtest || exit 1
mkdir -p gpurun_out/pk
timeout -k 10 900 env ANA_DIST_BACKEND=gloo python3 bench.py --gpus 8 --steps 2 --warmup 1 > gpurun_out/pk/gloo8.log 2>&1 || { tail -5 gpurun_out/pk/gloo8.log; exit 1; }
python3 - <<'PY'
import json
d=json.loads([l for l in open("gpurun_out/pk/gloo8.log") if l.startswith("{")][-1]); a=d["accuracy"]
print("gloo8", d["ms_per_step"], "spearman", a["spearman_mu_minus_sigma"], "records", a["records_dmu_median"], a["records_dmu_p99"], a["records_dmu_max"], "clamps", a["merge_clamp_hits"], "bytes", d["merge_ms"].get("bytes_per_rank"))
PY
for r in 1 2; do
  for nb in 8:300 8:600; do
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --force-merge --merges-per-step 8 --emulate-allreduce $nb > gpurun_out/pk/emu${nb/:/_}_$r.log 2>&1 || exit 1
    echo "emu $nb round $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pk/emu${nb/:/_}_$r.log)"
  done
done
