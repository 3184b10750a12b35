"""The worker's GPU path: a device-resident roster + per-batch graph replay.

The reference rates each batch of <= BATCHSIZE matches by loading the players
from MySQL, rating match after match in Python and committing the player rows
back (/root/reference/worker.py:169-199, rater.py:108-169).  Rebuilding a
device roster from those objects for every batch costs more than the rating
itself, so ``ENGINE=native`` keeps the player table ON THE DEVICE across
batches:

* ``ResidentRoster``: the ``Roster`` tensors (128 B per player) plus an
  ``api_id -> row`` map that grows when a batch brings players it has not seen
  (their stored ratings are uploaded once, with one H2D copy per batch;
  capacity doubles when full).  The worker is then the owner of the ratings it
  writes: rows are never re-read from the store (``RESIDENT=false`` restores
  the rebuild-per-batch path for deployments that share the table with other
  writers -- the reference's replicas race on those rows anyway,
  worker.py:174-194);
* each batch is encoded columnarly into the stream layout and rated by ONE
  HIP-graph replay per team size (ops/graph.py; copy -> schedule -> executor),
  all graphs sharing the roster's epoch clock.  ``DOTELEMETRY`` launches the
  fused rating + telemetry executor eagerly on the same clock;
* only the batch's outputs (one packed 128-B row per match) and the batch's
  player rows come back to the host, and only the fields the reference writes
  are set on the objects (rater.py:103-105,141,151-169);
* a failed batch (exception after rating, QUARANTINE=false errors, a failed
  commit) is rolled back on the device too: the batch's rows are snapshotted
  before the launch and restored by ``rollback``.

On the CPU the same class rates through the C++ host mirror (no graphs).
"""
from __future__ import annotations

import math
from operator import attrgetter
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..config import MODES, TRACK_COLUMNS
from ..ops import rate as R
from ..utils.trace import trace_range
from .objects import STAT_COLUMNS, Match, ParticipantStats

RATING_COLS = tuple(c + s for c in TRACK_COLUMNS for s in ("_mu", "_sigma"))
ATTR_COLS = ("rank_points_ranked", "rank_points_blitz", "skill_tier")
_get_ratings = attrgetter(*RATING_COLS)
_get_attrs = attrgetter(*ATTR_COLS)
MODE_INDEX = {m: k for k, m in enumerate(MODES)}
MAX_TEAM = 5
_MU = [c + "_mu" for c in TRACK_COLUMNS]
_SIG = [c + "_sigma" for c in TRACK_COLUMNS]


def _f(x: float) -> Optional[float]:
    return None if math.isnan(x) else x


class ResidentRoster:
    """Device roster of every player the worker has seen, keyed by api id."""

    def __init__(self, device, capacity: int = 1 << 16):
        self.device = torch.device(device)
        self.roster = R.Roster.empty(max(1, int(capacity)), self.device)
        self.rows: Dict[str, int] = {}
        self.by_key = np.full(0, -1, dtype=np.int64)  # integer store key -> row (columnar stores)
        self.n = 0
        self.generation = 0  # bumped when the tensors move (graphs must be re-captured)

    def rows_for_keys(self, keys: np.ndarray, fetch) -> np.ndarray:
        """Rows of integer store keys (unique); ``fetch(new_keys)`` returns the
        stored (ratings [n, 14], attributes [n, 3]) of keys not seen before."""
        keys = np.asarray(keys, dtype=np.int64)
        if keys.size == 0:
            return keys
        top = int(keys.max()) + 1
        if top > self.by_key.size:
            grown = np.full(max(top, 2 * self.by_key.size), -1, dtype=np.int64)
            grown[:self.by_key.size] = self.by_key
            self.by_key = grown
        rows = self.by_key[keys]
        new = rows < 0
        if new.any():
            nk = keys[new]
            # fetch and upload first: a failing fetch must not leave keys mapped to
            # rows that were never written (the next batch would reuse the rows)
            ratings, attrs = fetch(nk)
            nr = self.n + np.arange(nk.size)
            self._upload_arrays(np.asarray(ratings, dtype=np.float64), np.asarray(attrs, dtype=np.float64))
            self.by_key[nk] = nr
            rows[new] = nr
        return rows

    def staging(self, k: int) -> torch.Tensor:
        """Host buffer [k, 36] for ``upload_staged`` (pinned on a GPU)."""
        return torch.empty((k, 36), dtype=torch.float32, pin_memory=self.device.type == "cuda")

    def upload_staged(self, buf: torch.Tensor) -> None:
        """Append rows staged as [k, 36] = state row (32) + attributes (4): one
        asynchronous H2D copy."""
        base, k = self.n, buf.shape[0]
        if base + k > self.capacity:
            self._grow(base + k)
        dev = buf.to(self.device, non_blocking=True)
        _copy_rows(self.roster.state[base:base + k], dev[:, :32])
        _copy_rows(self.roster.attrs[base:base + k], dev[:, 32:])
        self.n = base + k

    def _upload_arrays(self, vals: np.ndarray, attrs: np.ndarray) -> None:
        """Append rows from stored ratings [k, 14] (NaN = NULL) and attributes [k, 3]."""
        k = vals.shape[0]
        buf = self.staging(k)
        st = buf.numpy()
        st[:, 0:32] = 0.0
        mu = vals[:, 0::2]
        st[:, 0:28:4] = mu
        st[:, 2:28:4] = np.where(np.isnan(mu), np.nan, vals[:, 1::2])
        st[:, 28:32:2] = np.nan
        st[:, 32:35] = attrs
        st[:, 35] = 0.0
        self.upload_staged(buf)

    @property
    def capacity(self) -> int:
        return self.roster.num_players

    def rows_for(self, players: Sequence) -> List[int]:
        """Row of every player object (uploading the ones not seen before)."""
        rows, new, fresh = [], [], {}
        get = self.rows.get
        for pl in players:
            r = get(pl.api_id)
            if r is None:
                r = fresh.get(pl.api_id)
                if r is None:
                    r = self.n + len(new)
                    fresh[pl.api_id] = r
                    new.append(pl)
            rows.append(r)
        if new:
            self._upload(new)  # the map only learns rows that were written
            self.rows.update(fresh)
        return rows

    def forget(self, api_ids) -> int:
        """Drop cached rows of these players (rated elsewhere, e.g. by the Python
        engine): their next batch re-reads them from the store.  The rows
        themselves stay allocated (orphaned) until the roster is rebuilt."""
        n = 0
        for a in api_ids:
            if self.rows.pop(a, None) is not None:
                n += 1
        return n

    def reset(self) -> None:
        """Forget every cached player (RESIDENT=false on a columnar store: each batch
        re-reads its players from the store, so other replicas' commits are seen).
        The rows are reused from 0; the tensors stay where they are."""
        self.rows.clear()
        self.by_key[:] = -1
        self.n = 0

    def _grow(self, need: int) -> None:
        cap = self.capacity
        while cap < need:
            cap *= 2
        bigger = R.Roster.empty(cap, self.device)
        bigger.state[:self.n].copy_(self.roster.state[:self.n])
        bigger.attrs[:self.n].copy_(self.roster.attrs[:self.n])
        self.roster = bigger
        self.generation += 1

    def _upload(self, new: Sequence) -> None:
        k = len(new)
        vals = np.array([_get_ratings(pl) for pl in new], dtype=np.float64).reshape(k, len(RATING_COLS))
        attrs = np.array([_get_attrs(pl) for pl in new], dtype=np.float64).reshape(k, 3)
        self._upload_arrays(vals, attrs)


def team_size(matches: Sequence[Match]) -> int:
    k = 1
    for m in matches:
        for r in m.rosters[:2]:
            n = len(r.participants)
            if n > k:
                k = n
    return k


def encode(matches: Sequence[Match], row_of: Dict[int, int], K: int) -> torch.Tensor:
    """``[M, 2K+2]`` int32 records (csrc/common.h layout) from object matches;
    ``row_of`` maps ``id(player object)`` to its roster row."""
    S = 2 * K
    out = np.full((len(matches), S + 2), -1, dtype=np.int64)
    for i, m in enumerate(matches):
        rosters = m.rosters
        nr = len(rosters)
        row = out[i]
        afk = 0
        k = 0
        n = [0, 0]
        for ri in range(min(nr, 2)):
            parts = rosters[ri].participants
            n[ri] = len(parts)
            off = ri * K
            for pos, p in enumerate(parts):
                if pos < K:
                    row[off + pos] = row_of[id(p.player[0])]
                if p.went_afk == 1:
                    afk |= 1 << min(k, 23)
                k += 1
        for ri in range(2, nr):
            for p in rosters[ri].participants:
                if p.went_afk == 1:
                    afk |= 1 << 23
        w0 = nr > 0 and bool(rosters[0].winner)
        w1 = nr > 1 and bool(rosters[1].winner)
        row[S] = (MODE_INDEX.get(m.game_mode, 255) | (min(n[0], 255) << 8) | (min(n[1], 255) << 16)
                  | (min(nr, 255) << 24))
        row[S + 1] = (1 if w0 else 0) | (2 if w1 else 0) | (4 if afk else 0) | ((afk & 0xffffff) << 8)
    return torch.from_numpy(out.astype(np.uint32).view(np.int32))


class ResidentBatchRater:
    """``ENGINE=native`` batch rater over a ``ResidentRoster`` (see module doc)."""

    def __init__(self, rater: Optional[R.BatchRater] = None, device=None, capacity: int = 500,
                 roster_capacity: int = 1 << 16, graphs: bool = True):
        self.rater = rater or R.BatchRater()
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.resident = ResidentRoster(self.device, roster_capacity)
        self.capacity = int(capacity)
        self.use_graphs = graphs and self.device.type == "cuda"
        self._graphs: Dict[int, object] = {}
        self._clock = None
        self._generation = -1
        self._undo = None  # (rows, saved state rows) of the last batch

    def supports(self, matches: Sequence[Match]) -> bool:
        return team_size(matches) <= MAX_TEAM

    # ------------------------------------------------------------ graphs
    def _graph(self, K: int, m: int):
        from ..ops.graph import EpochClock, GraphRater

        if self._generation != self.resident.generation:  # the roster moved
            self._graphs.clear()
            self._clock = EpochClock(self.resident.roster)
            self._generation = self.resident.generation
        if m > self.capacity:
            return None
        g = self._graphs.get(K)
        if g is None:
            g = GraphRater(self.resident.roster, K, self.capacity, self.rater, clock=self._clock)
            self._graphs[K] = g
        return g

    # ------------------------------------------------------------ rating
    def rate(self, matches: Sequence[Match], telemetry=None) -> List[int]:
        if not matches:
            return []
        K = team_size(matches)
        if K > MAX_TEAM:
            raise ValueError("teams of %d players exceed the batched engine (max %d)" % (K, MAX_TEAM))
        players, row_of = [], {}
        for m in matches:
            for r in m.rosters[:2]:
                for p in r.participants:
                    pl = p.player[0]
                    if id(pl) not in row_of:
                        row_of[id(pl)] = -1
                        players.append(pl)
        rows = self.resident.rows_for(players)
        for pl, r in zip(players, rows):
            row_of[id(pl)] = r
        rec = encode(matches, row_of, K).to(self.device, non_blocking=True)
        roster = self.resident.roster
        idx = torch.tensor(rows, dtype=torch.int64).to(self.device, non_blocking=True)
        self._undo = (idx, _gather_rows(roster.state, idx)) if rows else None
        stats = None
        if telemetry is not None:
            from ..ops.telemetry import allocate_stats, make_telemetry
            tel = make_telemetry(telemetry, rec, K, ids=[m.api_id for m in matches])
            stats = allocate_stats(len(matches), K, self.device)
            res = self._eager(rec, K, (tel.evoff, tel.events, stats))
        else:
            g = self._graph(K, len(matches)) if self.use_graphs else None
            res = g.rate(rec) if g is not None else self._eager(rec, K, None)
        packed = res.packed.cpu().numpy() if res.packed is not None else None
        final = _gather_rows(roster.state, idx).cpu().numpy() if rows else None
        st = self._write_back(matches, res, packed, K, row_of, final, rows)
        if stats is not None:
            _write_stats(matches, stats, K, st)
        if self.device.type == "cuda":
            self.rater.check_errors(self.device)
        return st

    def rate_batch(self, batch, fetch, telemetry=None, stage=None) -> np.ndarray:
        """Rate a columnar ``MatchBatch`` (runtime/columnar.py) in order and fill
        its result columns; ``fetch(keys)`` gives the stored ratings of players
        the resident roster has not seen.  Returns the status per match."""
        return self.finish_batch(self.launch_batch(batch, fetch, telemetry, stage))

    def launch_batch(self, batch, fetch, telemetry=None, stage=None) -> "PendingBatch":
        """First half of ``rate_batch``: encode, upload, launch and enqueue the
        copies back into pinned buffers -- nothing waits on the device, so the
        worker can prepare the next batch (or finish the previous one) while
        this one rates.  Launches are stream-ordered: a batch launched after
        another rates from that one's results.  ``stage(keys, out)`` (optional,
        the columnar store's) writes new players' upload rows directly instead
        of ``fetch``."""
        M, K = len(batch), batch.K
        if K > MAX_TEAM:
            raise ValueError("teams of %d players exceed the batched engine (max %d)" % (K, MAX_TEAM))
        if M == 0:
            return PendingBatch(batch, K)
        C = R.native()
        t = torch.from_numpy
        res_ = self.resident
        with trace_range("rate.rows"):
            top = batch.key_bound if batch.key_bound is not None else int(batch.player.max()) + 1
            if top > res_.by_key.size:
                grown = np.full(max(top, 2 * res_.by_key.size), -1, dtype=np.int64)
                grown[:res_.by_key.size] = res_.by_key
                res_.by_key = grown
            # records, the batch's unique players (first-seen order) and their resident
            # rows; players not resident yet were given the next rows (csrc/batch_host.cpp)
            rec_c, uniq_t, rows_t, pos_t, new_t = C.batch_encode(
                t(batch.player), t(batch.mode), t(batch.n), t(batch.nrosters), t(batch.winner),
                t(batch.afk), t(res_.by_key), res_.n)
            if new_t.numel():
                nk = new_t.numpy()
                try:
                    if stage is not None:
                        buf = res_.staging(nk.size)
                        stage(new_t, buf)
                        res_.upload_staged(buf)
                    else:
                        ratings, attrs = fetch(nk)
                        res_._upload_arrays(np.asarray(ratings, dtype=np.float64),
                                            np.asarray(attrs, dtype=np.float64))
                except BaseException:  # the map must not keep rows that were never written
                    res_.by_key[nk] = -1
                    raise
        with trace_range("rate.encode_h2d"):
            rec_t = rec_c.to(self.device, non_blocking=True)
            roster = res_.roster
            idx = rows_t.to(self.device, non_blocking=True)
            undo = (idx, _gather_rows(roster.state, idx)) if rows_t.numel() else None
        self._undo = undo
        p = PendingBatch(batch, K, pos_t, uniq_t, undo=undo)
        if telemetry is not None:
            from ..ops.telemetry import allocate_stats, make_telemetry
            tel = make_telemetry(telemetry, rec_t, K, ids=batch.ids)
            p.stats = allocate_stats(M, K, self.device)
            res = self._eager(rec_t, K, (tel.evoff, tel.events, p.stats))
        else:
            with trace_range("rate.launch"):
                g = self._graph(K, M) if self.use_graphs else None
                res = g.rate(rec_t) if g is not None else self._eager(rec_t, K, None)
        # outputs, the players' final rows and the error flags: asynchronous
        # copies into pinned buffers, one event to wait on
        p.packed = _to_host(res.packed)
        p.final = _to_host(_gather_rows(roster.state, idx)) if rows_t.numel() else None
        if self.device.type == "cuda":
            p.flags = _to_host(self.rater.error_flags(self.device))
            if p.stats is not None:
                p.stats = _to_host(p.stats)
            p.event = torch.cuda.Event()
            p.event.record()
        return p

    def finish_batch(self, p: "PendingBatch") -> np.ndarray:
        """Second half of ``rate_batch``: wait for the batch's copies and fill its
        result columns (csrc/batch_host.cpp batch_finish)."""
        batch, K = p.batch, p.K
        M = len(batch)
        if M == 0:
            batch.status = np.zeros(0, dtype=np.uint8)
            return batch.status
        with trace_range("rate.d2h"):
            if p.event is not None:
                p.event.synchronize()
                self.rater.raise_flags(p.flags)
        with trace_range("rate.finish"):
            empty = torch.zeros(0, dtype=torch.float32)
            status_t, quality_t, fields_t, fk_t, fv_t, ft_t = R.native().batch_finish(
                p.packed, p.final if p.final is not None else empty, torch.from_numpy(batch.mode), p.pos,
                p.uniq, K)
        status = status_t.numpy()
        batch.status = status
        batch.quality = quality_t.numpy()
        batch.fields = fields_t.numpy()
        batch.s_mu, batch.s_sig, batch.delta, batch.m_mu, batch.m_sig = batch.fields
        if p.stats is not None:
            batch.stats = p.stats.double().numpy().reshape(M, 2, K, -1)
        batch.final_keys, batch.final, batch.final_tracks = fk_t.numpy(), fv_t.numpy(), ft_t.numpy()
        return status

    def _eager(self, rec, K, telemetry):
        if self.device.type != "cuda":
            return self.rater.rate(self.resident.roster, rec, K, telemetry=telemetry)
        if self._clock is None or self._generation != self.resident.generation:
            self._graph(K, self.capacity + 1)  # (re)creates the clock only
        self._clock.before_launch()
        res = self.rater.rate(self.resident.roster, rec, K, telemetry=telemetry, check=False,
                              epoch_dev=self._clock.epoch)
        self._clock.launched()
        return res

    def rollback(self, pending: Optional["PendingBatch"] = None) -> None:
        """Undo the last batch (or ``pending``) on the device roster (the store
        rolled back).  With several batches launched, undo the latest first."""
        undo = self._undo if pending is None else pending.undo
        if pending is not None:
            pending.undo = None
        if undo is not None:
            idx, saved = undo
            # the snapshot may predate an EpochClock reset (before_launch renumbers
            # epochs after 255 launches): restore values with zeroed tag words, which
            # no launch's epoch ever matches, as unpack_rows does
            saved = saved.clone()
            saved[:, 1::2] = 0.0
            _scatter_rows(self.resident.roster.state, idx, saved)
        if self._undo is undo:
            self._undo = None

    def commit(self) -> None:
        self._undo = None

    @staticmethod
    def _write_back(matches, res, packed, K, row_of, final, rows) -> List[int]:
        S = 2 * K
        if packed is not None:
            st = packed.view(np.uint8)[:, 4 * (5 * S + 1)]
            q = packed[:, 5 * S].astype(np.float64).tolist()
            s_mu = packed[:, 0:S].astype(np.float64).tolist()
            s_sig = packed[:, S:2 * S].astype(np.float64).tolist()
            dl = packed[:, 2 * S:3 * S].astype(np.float64).tolist()
            m_mu = packed[:, 3 * S:4 * S].astype(np.float64).tolist()
            m_sig = packed[:, 4 * S:5 * S].astype(np.float64).tolist()
        else:
            st = res.status.cpu().numpy()
            q = res.quality.cpu().double().tolist()
            s_mu, s_sig, dl, m_mu, m_sig = (t.cpu().double().tolist()
                                            for t in (res.s_mu, res.s_sig, res.delta, res.m_mu, res.m_sig))
        status = [int(x) for x in st.tolist()]
        touched: Dict[int, set] = {}
        skip = set(R.ERROR_STATUSES) | {R.UNSUPPORTED_MODE, R.NOT_PROCESSED}
        for i, m in enumerate(matches):
            s = status[i]
            if s in skip:
                continue
            if s == R.AFK or s == R.INVALID_ROSTERS:
                m.trueskill_quality = 0
                for p in m.participants:
                    p.participant_items[0].any_afk = True
                continue
            mode = MODE_INDEX[m.game_mode]
            cmu, csig = _MU[1 + mode], _SIG[1 + mode]
            m.trueskill_quality = q[i]
            for p in m.participants:
                p.participant_items[0].any_afk = False
            smu, ssg, sdl, mmu, msg = s_mu[i], s_sig[i], dl[i], m_mu[i], m_sig[i]
            for ri, r in enumerate(m.rosters[:2]):
                off = ri * K
                for pos, p in enumerate(r.participants):
                    j = off + pos
                    p.trueskill_mu = smu[j]
                    p.trueskill_sigma = ssg[j]
                    p.trueskill_delta = sdl[j]
                    it = p.participant_items[0]
                    setattr(it, cmu, mmu[j])
                    setattr(it, csig, msg[j])
                    key = id(p.player[0])
                    t = touched.get(key)
                    if t is None:
                        touched[key] = t = set()
                    t.add(0)
                    t.add(1 + mode)
        if final is None or not touched:
            return status
        fin = final.astype(np.float64)
        by_id = {}
        for m in matches:
            for p in m.participants:
                by_id[id(p.player[0])] = p.player[0]
        pos_of = {r: k for k, r in enumerate(rows)}
        for key, tracks in touched.items():
            pl = by_id[key]
            row = fin[pos_of[row_of[key]]]
            for t in tracks:
                setattr(pl, _MU[t], _f(float(row[4 * t])))
                setattr(pl, _SIG[t], _f(float(row[4 * t + 2])))
        return status


class PendingBatch:
    """A launched columnar batch (``ResidentBatchRater.launch_batch``)."""

    def __init__(self, batch, K: int, pos=None, uniq=None, undo=None):
        self.batch, self.K, self.pos, self.uniq, self.undo = batch, K, pos, uniq, undo
        self.packed = self.final = self.flags = self.stats = self.event = None


# Row gathers / scatters / copies of the roster.  On the CPU (the host mirror) they go
# through numpy: torch's intra-op pool wakes every thread for a few thousand 128-B
# rows, which measured 30-120 ms per call on an 8-core host against 0.1 ms in numpy.
def _gather_rows(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    if t.device.type == "cpu":
        return torch.from_numpy(t.numpy()[idx.numpy()])
    return t.index_select(0, idx)


def _scatter_rows(t: torch.Tensor, idx: torch.Tensor, rows: torch.Tensor) -> None:
    if t.device.type == "cpu":
        t.numpy()[idx.numpy()] = rows.numpy()
    else:
        t.index_copy_(0, idx, rows)


def _copy_rows(dst: torch.Tensor, src: torch.Tensor) -> None:
    if dst.device.type == "cpu" and src.device.type == "cpu":
        dst.numpy()[...] = src.numpy()
    else:
        dst.copy_(src)


def _to_host(src: torch.Tensor) -> torch.Tensor:
    """``src`` on the host: on a GPU an asynchronous copy into pinned memory
    (PyTorch's caching host allocator recycles the buffers)."""
    if src.device.type != "cuda":
        return src.contiguous()
    out = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
    out.copy_(src, non_blocking=True)
    return out


def _write_stats(matches, stats: torch.Tensor, K: int, status) -> None:
    """participant_stats of every committed match (not the quarantined ones)."""
    st = stats.cpu().double().numpy()
    bad = set(R.ERROR_STATUSES) | {R.NOT_PROCESSED}
    for i, m in enumerate(matches):
        if int(status[i]) in bad:
            continue
        for ri, r in enumerate(m.rosters[:2]):
            for pos, p in enumerate(r.participants[:K]):
                vals = dict(zip(STAT_COLUMNS, (float(v) for v in st[i, ri * K + pos])))
                p.participant_stats = [ParticipantStats(p.api_id, **vals)]
