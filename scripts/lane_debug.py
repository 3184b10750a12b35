"""Debug the per-lane executor against the fp64 host mirror on small dense specs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from analyzer_amd.ops import rate as R  # noqa: E402
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_engine_host import SPECS  # noqa: E402

dev = torch.device("cuda:0")
for name in ["5v5_edge", "uneven_K4", "3v3", "1v1_empty"]:
    rspec, sspec, K = SPECS[name]
    roster = make_roster(rspec)
    rec = make_stream(sspec, 20000, rspec.num_players, K=K)
    host = roster.clone()
    rh = R.BatchRater(host_fp64=True).rate(host, rec, K)
    for impl in ("0", "1"):
        for local in ("1", "0"):
            os.environ["ANA_RATE_IMPL"] = impl
            os.environ["ANA_RATE_LOCAL"] = local
            ro = roster.to(dev)
            br = R.BatchRater()
            res = br.rate(ro, rec.to(dev), K, check=False)
            torch.cuda.synchronize()
            flags = br.error_flags(dev).cpu().tolist()
            st = res.status.cpu().numpy()
            bad = np.nonzero(st != rh.status.numpy())[0]
            dmu = np.abs(np.nan_to_num(res.s_mu.cpu().numpy() - rh.s_mu.numpy(), nan=0.0)).max(1)
            nanmis = (np.isnan(res.s_mu.cpu().numpy()) != np.isnan(rh.s_mu.numpy())).any(1)
            wrong = np.nonzero((dmu > 6e-3) | nanmis)[0]
            print(name, "impl", impl, "local", local, "flags", flags, "stale", br.stale_retries(dev),
                  "status mismatches", len(bad), bad[:5], "mu mismatches", len(wrong), wrong[:5], flush=True)
            if len(wrong):
                m = int(wrong[0])
                print("  first wrong match", m, "rec", rec[m].tolist(), "dev", res.s_mu.cpu()[m].tolist(),
                      "host", rh.s_mu[m].tolist(), "status", int(st[m]), int(rh.status[m]), flush=True)
