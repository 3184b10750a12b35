"""Time the schedule prepass alone (experiments on its kernels).

    python scripts/sched_time.py [MATCHES] [TEAM_SIZE]   (default 10M 3v3 over 1M players)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from analyzer_amd.ops.rate import BatchRater
from analyzer_amd.ops.synth import StreamSpec, make_stream
dev = torch.device("cuda:0")
M, P = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000, 1_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rec = make_stream(StreamSpec(team_size=K, seed=5), M, P, K=K, device=dev)
br = BatchRater()
ts = []
for i in range(6):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    br.schedule(rec, K, P)
    torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
print("schedule ms min %.3f median %.3f" % (min(ts), sorted(ts)[3]))
