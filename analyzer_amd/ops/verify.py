"""Numerical verification of the device executor against the fp64 host mirror.

The reference computes with 50-digit mpmath (/root/reference/rater.py:7-8);
the MI355X executor keeps fp32 state and uses the hardware reciprocal/sqrt paths
(build_ext.py ``-fapprox-func``).  SURVEY §4 item 2 gates a single match at
|d mu| <= 1e-3; over a window every player's rating is a chain of updates
(~60 per player for 10M 3v3 matches over 1M players), so rounding accumulates.
``verify_window`` measures exactly that at bench scale: it rates one window on
the device and the same window on the C++ host mirror in fp64 (csrc/host.cpp,
the same rate_core.h formulas instantiated for double) from the same roster,
and reports the worst deviations over every output record and over the final
roster.  The fp64 host mirror is itself pinned to the reference's numerics by
tests/test_models.py (SURVEY App. B goldens, fp64 oracle / mpmath).
"""
from __future__ import annotations

from typing import Dict

import torch

from .rate import BatchRater, RateResult, Roster


def _stats(a: torch.Tensor, b: torch.Tensor, rel: bool) -> Dict[str, float]:
    a = a.double().reshape(-1)
    b = b.double().reshape(-1)
    both = ~torch.isnan(a) & ~torch.isnan(b)
    d = (a[both] - b[both]).abs()
    if rel:
        d = d / b[both].abs().clamp_min(1e-30)
    out = {"n": int(both.sum()), "nan_mismatch": int((torch.isnan(a) != torch.isnan(b)).sum())}
    if d.numel():
        out["max"] = float(d.max())
        s = d if d.numel() <= 1 << 24 else d[torch.randperm(d.numel())[: 1 << 24]]
        out["p99"] = float(torch.quantile(s, 0.99))
        out["median"] = float(torch.quantile(s, 0.5))
    return out


def compare_results(dev_out: RateResult, host_out: RateResult, dev_roster: Roster,
                    host_roster: Roster) -> Dict[str, object]:
    d = {
        "status_mismatch": int((dev_out.status.cpu() != host_out.status).sum()),
        "out_shared_mu_abs": _stats(dev_out.s_mu.cpu(), host_out.s_mu, False),
        "out_shared_sigma_rel": _stats(dev_out.s_sig.cpu(), host_out.s_sig, True),
        "out_mode_mu_abs": _stats(dev_out.m_mu.cpu(), host_out.m_mu, False),
        "out_mode_sigma_rel": _stats(dev_out.m_sig.cpu(), host_out.m_sig, True),
        "out_delta_abs": _stats(dev_out.delta.cpu(), host_out.delta, False),
        "out_quality_abs": _stats(dev_out.quality.cpu(), host_out.quality, False),
    }
    ds, hs = dev_roster.state.cpu(), host_roster.state
    d["roster_mu_abs"] = _stats(ds[:, 0::4], hs[:, 0::4], False)
    d["roster_sigma_rel"] = _stats(ds[:, 2::4], hs[:, 2::4], True)
    return d


def verify_window(roster: Roster, rec: torch.Tensor, K: int) -> Dict[str, object]:
    """Rate ``rec`` from ``roster`` (left untouched) on its device and on the fp64
    host mirror; return the deviation statistics (see ``compare_results``)."""
    dev_roster = roster.clone()
    host_roster = Roster(roster.state.cpu().clone(), roster.attrs.cpu().clone(), epoch=0)
    dev_out = BatchRater().rate(dev_roster, rec, K)
    host_out = BatchRater(host_fp64=True).rate(host_roster, rec.cpu(), K)
    res = compare_results(dev_out, host_out, dev_roster, host_roster)
    res["matches"] = int(rec.shape[0])
    return res
