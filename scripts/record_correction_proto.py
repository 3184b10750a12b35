#!/usr/bin/env python3
"""Prototype of the causal record correction in plain torch (round 5): 8 ranks
simulated, records corrected by the exclusive prefix of raw fp32 messages; prints
the last window's record errors against exact sequential rating (usage: k)."""
import sys, torch
sys.path.insert(0, "/root/repo")
from analyzer_amd.parallel.sweep import SweepMerger
from analyzer_amd.parallel.accuracy import _q
from analyzer_amd.ops.rate import BatchRater
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
ranks, P, k = 8, 100000, int(sys.argv[1])
Mw = 1000000 // k; K = 3
rater = BatchRater()
base = make_roster(RosterSpec(num_players=P, seed=11, p_rated=0.3))
spec = StreamSpec(team_size=K, seed=12)
off = 0
for r in range(ranks):
    rater.rate(base, make_stream(spec, 1000000 // ranks, P, K=K, base=off), K); off += 1000000 // ranks
exact = base.clone(); approx = base.clone()
E = {"s_raw": [], "s_cor": [], "m_raw": [], "m_cor": [], "d_raw": []}
def nat_add(mu, sg, dpi, dtau):
    pi = 1.0 / sg.double() ** 2; tau = mu.double() * pi
    pi2 = pi + dpi.double(); tau2 = tau + dtau.double()
    return (tau2 / pi2).float(), (1.0 / pi2.sqrt()).float()
for w in range(k):
    shards = [make_stream(spec, Mw, P, K=K, base=off + (w * ranks + r) * Mw) for r in range(ranks)]
    out_e = [rater.rate(exact, sh, K) for sh in shards]
    mergers = [SweepMerger(P, "cpu", rater.cfg, comm_dtype="fp32", world_size=ranks) for _ in range(ranks)]
    rosters = [approx.clone() for _ in range(ranks)]
    outs = []
    for m, ro, sh in zip(mergers, rosters, shards):
        m.begin(ro); outs.append(rater.rate(ro, sh, K)); m.rated(); m.messages(ro)
    msgs = [m.buf.clone() for m in mergers]
    prefix = torch.zeros_like(msgs[0])
    last = w == k - 1
    for r in range(ranks):
        a, e = outs[r], out_e[r]
        ok = (a.status == 0) & (e.status == 0)
        idc = shards[r][:, :2 * K].long().clamp(0, P - 1)
        mode = (shards[r][:, 2 * K] & 0xFF).long().clamp(0, 5)
        smu, _ = nat_add(a.s_mu, a.s_sig, prefix[idc, 0], prefix[idc, 1])
        col = (2 * (1 + mode))[:, None].expand_as(idc)
        mmu, _ = nat_add(a.m_mu, a.m_sig, prefix[idc, col], prefix[idc, col + 1])
        if last:
            for key, x, y in (("s_raw", a.s_mu, e.s_mu), ("s_cor", smu, e.s_mu), ("m_raw", a.m_mu, e.m_mu), ("m_cor", mmu, e.m_mu), ("d_raw", a.delta, e.delta)):
                d = (x - y)[ok].abs(); E[key].append(d[~torch.isnan(d)])
        prefix = prefix + msgs[r]
    total = torch.stack(msgs).sum(0)
    for m, ro in zip(mergers, rosters):
        m.buf.copy_(total); m.decode(ro, into=m.start)
    approx.state.copy_(rosters[0].state)
print("k=%d last window: " % k + " | ".join("%s median %.2f p99 %.1f" % (key, _q(torch.cat(v), .5), _q(torch.cat(v), .99)) for key, v in E.items()))
