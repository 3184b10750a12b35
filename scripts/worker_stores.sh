# Worker throughput per store (scripts/worker_profile.py), run on the GPU box by scripts/gpu.sh worker.
set -o pipefail
for i in 1 2; do timeout -k 10 300 python scripts/worker_profile.py --synthetic 400000 --segments 8 --cprofile 0 > gpurun_out/worker_columnar_$i.json 2>&1 || exit 1; echo columnar $(grep -h "matches_per_s" gpurun_out/worker_columnar_$i.json | tr -d "\n "); done
timeout -k 10 300 python scripts/worker_profile.py --synthetic 200000 --segments 4 --cprofile 0 --pipeline true > gpurun_out/worker_columnar_pipelined.json 2>&1 || exit 1
rm -f gpurun_out/w*.db
timeout -k 10 300 python scripts/worker_profile.py --synthetic 20000 --cprofile 0 --store sqlite:///gpurun_out/w1.db > gpurun_out/worker_sqlite_native.json 2>&1 || exit 1
RESIDENT=true timeout -k 10 300 python scripts/worker_profile.py --synthetic 20000 --cprofile 0 --store sqlite:///gpurun_out/w2.db > gpurun_out/worker_sqlite_native_resident.json 2>&1 || exit 1
STORE_BACKEND=sqlalchemy timeout -k 10 300 python scripts/worker_profile.py --synthetic 20000 --cprofile 0 --store sqlite:///gpurun_out/w3.db > gpurun_out/worker_sqla_native.json 2>&1 || exit 1
STORE_BACKEND=sqlalchemy timeout -k 10 300 python scripts/worker_profile.py --synthetic 5000 --cprofile 0 --engine python --store sqlite:///gpurun_out/w4.db > gpurun_out/worker_sqla_python.json 2>&1 || exit 1
rm -f gpurun_out/w*.db
for f in gpurun_out/worker_*.json; do echo $f $(grep -h '"matches_per_s"' $f); done
