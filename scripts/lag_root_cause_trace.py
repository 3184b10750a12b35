import sys, torch
sys.path.insert(0, "/root/repo")
from analyzer_amd.parallel import accuracy as A
from analyzer_amd.parallel.sweep import SweepMerger
from analyzer_amd.ops.rate import BatchRater, RateResult
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
ranks, players, M, windows, K = 8, 100000, 125000, 4, 3
dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
rater = BatchRater()
base = make_roster(RosterSpec(num_players=players, seed=11, p_rated=0.3))
spec = StreamSpec(team_size=K, seed=12)
off = 0
for r in range(ranks):
    rater.rate(base, make_stream(spec, M, players, K=K, base=off), K); off += M
shard_sets = [[make_stream(spec, M, players, K=K, base=off + (w * ranks + r) * M) for r in range(ranks)] for w in range(windows)]
N = ranks
mergers = [SweepMerger(players, "cpu", rater.cfg, comm_dtype=dtype, world_size=N, lag=True) for _ in range(N)]
rosters = [base.clone() for _ in range(N)]
for m, ro in zip(mergers, rosters): m.begin(ro)
hist = []
for b, shards in enumerate(shard_sets):
    for r in range(N):
        mergers[r].begin(rosters[r]); rater.rate(rosters[r], shards[r], K); mergers[r].rated()
    X = [ro.state.clone() for ro in rosters]
    for m, ro in zip(mergers, rosters):
        m.lag_boundary(ro); m._has_sum = True
    if dtype == "fp32":
        msgs = [m.buf.clone() for m in mergers]
        total = torch.stack([m.buf for m in mergers]).sum(0)
        for m in mergers: m.buf.copy_(total)
        tot = total[:, 0]
        own = [x[:, 0] for x in msgs]
    else:
        own = [m.msg.float()[:, 0] for m in mergers]
        msg = torch.stack([m.msg.float() for m in mergers]).sum(0).to(mergers[0].msg.dtype)
        cnt = torch.stack([m.cnt for m in mergers]).sum(0)
        for m in mergers: m.msg.copy_(msg); m.cnt.copy_(cnt)
        tot = msg.float()[:, 0]
    C = mergers[0].start[:, :2].clone()
    hist.append((C, tot, own, [x[:, :4].clone() for x in X], [m.y[:, :2].clone() for m in mergers]))
    print("boundary", b, "min 1+sum dpi(shared)", float((1 + tot).min()), "count<0.05:", int(((1 + tot) < 0.05).sum()),
          "| C sigma min", float(C[:, 1].nan_to_num(1e9).min()))
bb = int(sys.argv[2]) if len(sys.argv) > 2 else len(hist) - 1
p = int(torch.argmin(1 + hist[bb][1]))
print("worst player", p)
for b, (C, tot, own, X, Y) in enumerate(hist):
    print(b, "C", C[p].tolist(), "sum dpi", float(tot[p]), "own dpi", [round(float(o[p]), 4) for o in own])
    print("   X mu,sig per rank", [(round(float(x[p, 0]), 1), round(float(x[p, 2]), 2)) for x in X])
    print("   Y per rank", [(round(float(y[p, 0]), 1), round(float(y[p, 1]), 2)) for y in Y])
