import sys, torch
sys.path.insert(0, "/root/repo")
from analyzer_amd.parallel.sweep import SweepMerger
from analyzer_amd.ops.rate import BatchRater
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
ranks, players, M, windows, K = 8, int(float(sys.argv[1])), int(float(sys.argv[2])), 4, 3
rater = BatchRater()
base = make_roster(RosterSpec(num_players=players, seed=11, p_rated=0.3))
spec = StreamSpec(team_size=K, seed=12)
off = 0
for r in range(ranks):
    rater.rate(base, make_stream(spec, M, players, K=K, base=off), K); off += M
sets = [[make_stream(spec, M, players, K=K, base=off + (w * ranks + r) * M) for r in range(ranks)] for w in range(windows)]
for lag in (True, False):
    mergers = [SweepMerger(players, "cpu", rater.cfg, comm_dtype="fp32", world_size=ranks, lag=lag) for _ in range(ranks)]
    rosters = [base.clone() for _ in range(ranks)]
    for m, ro in zip(mergers, rosters): m.begin(ro)
    for b, shards in enumerate(sets):
        for r in range(ranks):
            mergers[r].begin(rosters[r]); rater.rate(rosters[r], shards[r], K); mergers[r].rated()
        if lag:
            for m, ro in zip(mergers, rosters): m.lag_boundary(ro); m._has_sum = True
        else:
            for m, ro in zip(mergers, rosters): m.messages(ro)
        total = torch.stack([m.buf for m in mergers]).sum(0)
        C = mergers[0].start  # lag: C_b (the base the next sum lands on); plain: the window start
        pic = 1.0 / C[:, 1].double() ** 2
        ratio = (pic + total[:, 0].double()) / pic
        ok = ~torch.isnan(ratio)
        print("lag" if lag else "plain", "boundary", b, "min merged/base precision (shared) %.4f" % float(ratio[ok].min()),
              "players < 0.1: %d" % int((ratio[ok] < 0.1).sum()))
        for m in mergers: m.buf.copy_(total)
        if not lag:
            for m, ro in zip(mergers, rosters): m.decode(ro, into=m.start)
