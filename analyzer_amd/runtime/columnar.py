"""Columnar match batches and the columnar in-process store (worker ENGINE=native).

The reference's worker hands ORM objects to the rater one attribute at a time
(/root/reference/worker.py:176-192, rater.py:69-169); at GPU speed that object
traffic, not the rating, is the cost of a batch.  The native engine therefore
moves batches as columns end to end:

* ``MatchBatch``: one batch of matches in ``created_at`` order as arrays --
  game mode, roster sizes, winners, AFK mask, and per (match, roster, position)
  the store's participant and player keys; after rating, the outputs the
  reference writes (rater.py:103-105,141,151-169) as arrays of the same shape;
* ``ColumnarStore`` (``DATABASE_URI=columnar://``, also ``memory://``): the
  reference's tables kept as numpy columns.  ``load_batch`` / ``commit`` of a
  batch are a handful of vectorised gathers and scatters; ``load_matches``
  still materialises the object graph for ``ENGINE=python`` (and writes it back
  at commit), so both engines run on the same store;
* ``SqliteSession.load_batch`` (runtime/store.py) builds the same batch from
  three SELECTs and writes it back with ``executemany``.

Semantics are the object path's: outputs of unsupported-mode and error matches
are not written; AFK / invalid matches get quality 0 and ``any_afk`` on every
participant; rated matches write every participant and item and the players'
final ratings.  Writes become visible at ``commit`` only; ``rollback`` drops
them.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..config import MODES, TRACK_COLUMNS
from ..ops.native import native
from .objects import (STAT_COLUMNS, Match, Participant, ParticipantItems, ParticipantStats, Player,
                      Roster)

MODE_INDEX = {m: k for k, m in enumerate(MODES)}
UNSUPPORTED = 255
PLAYER_COLS = tuple(c + s for c in TRACK_COLUMNS for s in ("_mu", "_sigma"))      # 14
ITEM_COLS = tuple(c + s for c in TRACK_COLUMNS[1:] for s in ("_mu", "_sigma"))    # 12
ATTR_COLS = ("rank_points_ranked", "rank_points_blitz", "skill_tier")
NAN = float("nan")

# status codes (csrc/common.h; ops/rate.py)
RATED, AFK, INVALID = 0, 1, 2


def _nan(x) -> float:
    return NAN if x is None else float(x)


def _opt(x: float):
    return None if x != x else float(x)


@dataclass
class MatchBatch:
    """One worker batch as columns (matches in ``created_at`` order)."""

    ids: List[str]
    mode: np.ndarray            # [M] engine mode index, 255 = unsupported
    nrosters: np.ndarray        # [M]
    n: np.ndarray               # [M, 2] sizes of the first two rosters
    winner: np.ndarray          # [M, 2] bool (None counts as a loss, rater.py:144)
    afk: np.ndarray             # [M] AFK bit mask (csrc/common.h meta1 layout)
    player: np.ndarray          # [M, 2, K] store player key (int row) or -1
    part: np.ndarray            # [M, 2, K] store participant key (int row) or -1
    rows: Optional[np.ndarray] = None          # store match rows (columnar store)
    player_names: Optional[List[str]] = None   # player api id per key (SQL stores)
    extra_parts: Dict[int, List[int]] = field(default_factory=dict)  # rosters >= 2 of match i
    # results (ResidentBatchRater.rate_batch)
    status: Optional[np.ndarray] = None        # [M] uint8
    quality: Optional[np.ndarray] = None       # [M]
    s_mu: Optional[np.ndarray] = None          # [M, 2, K] shared mu / sigma / delta, mode mu / sigma
    s_sig: Optional[np.ndarray] = None
    delta: Optional[np.ndarray] = None
    m_mu: Optional[np.ndarray] = None
    m_sig: Optional[np.ndarray] = None
    stats: Optional[np.ndarray] = None         # [M, 2, K, 8] telemetry (DOTELEMETRY)
    final_keys: Optional[np.ndarray] = None    # [U] player keys of rated matches
    final: Optional[np.ndarray] = None         # [U, 14] their final (mu, sigma) per track
    final_tracks: Optional[np.ndarray] = None  # [U, 7] the tracks the batch wrote
    fields: Optional[np.ndarray] = None        # [5, M, 2, K] backing of s_mu .. m_sig (native finish)
    key_bound: Optional[int] = None            # every player key is below this (columnar store)

    @property
    def K(self) -> int:
        return int(self.player.shape[2])

    def __len__(self) -> int:
        return len(self.ids)

    def record_meta(self) -> Tuple[np.ndarray, np.ndarray]:
        """(meta0, meta1) words of the stream records (csrc/common.h)."""
        n = np.minimum(self.n, 255).astype(np.int64)
        m0 = (self.mode.astype(np.int64) | (n[:, 0] << 8) | (n[:, 1] << 16)
              | (np.minimum(self.nrosters, 255).astype(np.int64) << 24))
        afk = self.afk.astype(np.int64)
        m1 = (self.winner[:, 0].astype(np.int64) | (self.winner[:, 1].astype(np.int64) << 1)
              | ((afk != 0).astype(np.int64) << 2) | ((afk & 0xffffff) << 8))
        return m0, m1


def afk_mask(n: np.ndarray, afk0: np.ndarray, afk1: np.ndarray) -> np.ndarray:
    """AFK bit mask over the first two rosters: participant k (roster 0 first) sets
    bit min(k, 23) (runtime/objects.encode_matches)."""
    M, K = afk0.shape
    mask = np.zeros(M, dtype=np.int64)
    pos = np.arange(K)
    for p in range(K):
        mask |= np.where(afk0[:, p], np.int64(1) << min(p, 23), 0)
        k1 = np.minimum(n[:, 0] + p, 23)
        mask |= np.where(afk1[:, p], np.left_shift(np.int64(1), k1), 0)
    del pos
    return mask


def stats_mask(status: np.ndarray) -> np.ndarray:
    """Matches whose telemetry stats are written: every one that is committed
    (rated, AFK, invalid rosters, unsupported mode) -- not the quarantined ones."""
    from ..ops import rate as R

    return ~np.isin(status, list(R.ERROR_STATUSES) + [R.NOT_PROCESSED])


def touched_players(batch: MatchBatch) -> np.ndarray:
    """Player keys of the batch's rated matches (their final ratings are written)."""
    rated = batch.status == RATED
    keys = batch.player[rated].reshape(-1)
    return np.unique(keys[keys >= 0])


# ---------------------------------------------------------------- growable columns
class _Cols:
    """Row-growable set of equally long numpy columns."""

    def __init__(self, **spec):
        self._spec = spec  # name -> (trailing shape, dtype, fill)
        self.n = 0
        self._cap = 0
        for name, (shape, dtype, fill) in spec.items():
            setattr(self, name, np.full((0,) + shape, fill, dtype=dtype))

    def append(self, **vals) -> np.ndarray:
        k = len(next(iter(vals.values())))
        need = self.n + k
        if need > self._cap:
            cap = max(need, 2 * self._cap, 1024)
            for name, (shape, dtype, fill) in self._spec.items():
                old = getattr(self, name)
                new = np.full((cap,) + shape, fill, dtype=dtype)
                new[:self.n] = old[:self.n]
                setattr(self, name, new)
            self._cap = cap
        for name, v in vals.items():
            getattr(self, name)[self.n:need] = v
        rows = np.arange(self.n, need)
        self.n = need
        return rows


class ColumnarStore:
    """The reference's tables as numpy columns (see the module doc)."""

    columnar_batches = True  # sessions build MatchBatch columns (load_batch / fetch_players)

    # a session writes only at commit and a batch's load reads match structure and
    # the stored ratings of players no earlier batch touched, so the pipelined
    # worker may load batch i+1 while batch i's session is still open
    concurrent_sessions = True

    def __init__(self):
        self.players = _Cols(rating=((14,), np.float64, NAN), attr=((3,), np.float64, NAN))
        self.pl_ids: List[str] = []
        self.pl_index: Dict[str, int] = {}
        self.matches = _Cols(mode=((), np.int16, UNSUPPORTED), created=((), np.float64, 0.0),
                             quality=((), np.float64, NAN), r0=((), np.int64, 0), nr=((), np.int32, 0))
        self.m_ids: List[str] = []
        self.m_mode_name: List[str] = []
        self.m_index: Dict[str, int] = {}
        self.rosters = _Cols(winner=((), np.int8, -1), p0=((), np.int64, 0), np_=((), np.int32, 0))
        self.r_ids: List[str] = []
        self.parts = _Cols(player=((), np.int64, -1), afk=((), np.int8, -1), tier=((), np.float64, NAN),
                           ts=((3,), np.float64, NAN), i_afk=((), np.int8, 0),
                           i_rating=((12,), np.float64, NAN), stats=((8,), np.float64, NAN))
        self.p_ids: List[str] = []
        self.i_ids: List[str] = []
        self.p_index: Dict[str, int] = {}
        self.assets_by_match: Dict[str, List[str]] = {}
        self.commits = 0
        self._mkey = None  # native KeyIndex over m_ids (built on first batch lookup)

    def __getstate__(self):  # copies rebuild the native index
        d = dict(self.__dict__)
        d["_mkey"] = None
        return d

    def match_rows(self, ids: List) -> np.ndarray:
        """Store rows of match api ids (str or bytes), -1 where absent: one batched
        native lookup (csrc/batch_host.cpp KeyIndex), kept in step with m_ids."""
        if self._mkey is None:
            self._mkey = native().KeyIndex()
        k = len(self._mkey)
        if k < len(self.m_ids):
            try:
                self._mkey.add(self.m_ids[k:], k)
            except Exception:
                self._mkey = None  # rebuilt from m_ids on the next lookup, never left short
                raise
        return self._mkey.lookup(ids).numpy()

    # ------------------------------------------------------------- loading
    def add_players(self, players: Iterable[Player]) -> None:
        players = [p for p in players]
        new = [p for p in players if p.api_id not in self.pl_index]
        for p in players:  # replace existing rows in place
            r = self.pl_index.get(p.api_id)
            if r is not None:
                self.players.rating[r] = [_nan(getattr(p, c)) for c in PLAYER_COLS]
                self.players.attr[r] = [_nan(getattr(p, c)) for c in ATTR_COLS]
        if not new:
            return
        rating = np.array([[_nan(getattr(p, c)) for c in PLAYER_COLS] for p in new], dtype=np.float64)
        attr = np.array([[_nan(getattr(p, c)) for c in ATTR_COLS] for p in new], dtype=np.float64)
        rows = self.players.append(rating=rating, attr=attr)
        for p, r in zip(new, rows):
            self.pl_index[p.api_id] = int(r)
            self.pl_ids.append(p.api_id)

    def add_player_arrays(self, ids: Sequence[str], rating: np.ndarray, attr: np.ndarray) -> None:
        """Bulk insert of new players (synthetic populate)."""
        rows = self.players.append(rating=rating, attr=attr)
        for a, r in zip(ids, rows):
            self.pl_index[a] = int(r)
        self.pl_ids.extend(ids)

    def add_matches(self, matches: Iterable[Match]) -> None:
        for m in matches:
            if m.api_id in self.m_index:
                raise ValueError("match %s already stored" % m.api_id)
            for r in m.rosters:
                for p in r.participants:
                    if p.player[0].api_id not in self.pl_index:
                        self.add_players([p.player[0]])
            r0 = self.rosters.n
            for r in m.rosters:
                p0 = self.parts.n
                ps = r.participants
                self.parts.append(
                    player=np.array([self.pl_index[p.player[0].api_id] for p in ps], dtype=np.int64),
                    afk=np.array([-1 if p.went_afk is None else int(p.went_afk) for p in ps], dtype=np.int8),
                    tier=np.array([_nan(p.skill_tier) for p in ps], dtype=np.float64),
                    ts=np.array([[_nan(p.trueskill_mu), _nan(p.trueskill_sigma), _nan(p.trueskill_delta)]
                                 for p in ps], dtype=np.float64).reshape(len(ps), 3),
                    i_afk=np.array([-1 if p.participant_items[0].any_afk is None
                                    else int(bool(p.participant_items[0].any_afk)) for p in ps], dtype=np.int8),
                    i_rating=np.array([[_nan(getattr(p.participant_items[0], c)) for c in ITEM_COLS]
                                       for p in ps], dtype=np.float64).reshape(len(ps), 12))
                for p in ps:
                    self.p_index[p.api_id] = len(self.p_ids)
                    self.p_ids.append(p.api_id)
                    self.i_ids.append(p.participant_items[0].api_id or p.api_id)
                self.rosters.append(winner=np.array([-1 if r.winner is None else int(bool(r.winner))],
                                                    dtype=np.int8),
                                    p0=np.array([p0]), np_=np.array([len(ps)]))
                self.r_ids.append(r.api_id)
            row = self.matches.append(mode=np.array([MODE_INDEX.get(m.game_mode, UNSUPPORTED)]),
                                      created=np.array([float(m.created_at)]),
                                      quality=np.array([_nan(m.trueskill_quality)]),
                                      r0=np.array([r0]), nr=np.array([len(m.rosters)]))[0]
            self.m_index[m.api_id] = int(row)
            self.m_ids.append(m.api_id)
            self.m_mode_name.append(m.game_mode)

    def add_stream(self, rec: np.ndarray, K: int, player_ids: Sequence[str], base: int = 0,
                   prefix: str = "m") -> List[str]:
        """Bulk insert of a synthetic stream (records of csrc/common.h layout,
        player slots already store player rows); api ids / created_at as
        runtime/objects.matches_from_stream gives them."""
        rec = np.asarray(rec, dtype=np.int64)
        M = rec.shape[0]
        S = 2 * K
        m0 = rec[:, S] & 0xffffffff
        m1 = rec[:, S + 1] & 0xffffffff
        mode = m0 & 0xff
        n0, n1, nr = (m0 >> 8) & 0xff, (m0 >> 16) & 0xff, (m0 >> 24) & 0xff
        afkm = (m1 >> 8) & 0xffffff
        mids = ["%s%d" % (prefix, base + i) for i in range(M)]
        # reject duplicates before anything is written (add_matches does too): the
        # native match index (match_rows) must stay in step with m_ids
        if len(set(mids)) != M or any(a in self.m_index for a in mids):
            raise ValueError("add_stream: a match api id is already stored (prefix %r, base %d)" % (prefix, base))
        # rosters: the first two carry players, any further ones are empty
        r_first = self.rosters.n + np.concatenate([[0], np.cumsum(nr)[:-1]])
        nparts = n0 + n1
        p_first = self.parts.n + np.concatenate([[0], np.cumsum(nparts)[:-1]])
        # participants in order: roster 0 positions, then roster 1
        pl, afk, pids = [], [], []
        for i in range(M):
            k = 0
            for ri, n in ((0, n0[i]), (1, n1[i])):
                for pos in range(n):
                    pl.append(rec[i, ri * K + pos])
                    afk.append((afkm[i] >> k) & 1)
                    pids.append("%s%dp%d" % (prefix, base + i, k))
                    k += 1
        N = len(pl)
        self.parts.append(player=np.array(pl, dtype=np.int64), afk=np.array(afk, dtype=np.int8),
                          tier=np.full(N, NAN), ts=np.full((N, 3), NAN), i_afk=np.zeros(N, np.int8),
                          i_rating=np.full((N, 12), NAN))
        for a in pids:
            self.p_index[a] = len(self.p_ids)
            self.p_ids.append(a)
        self.i_ids.extend(pids)
        rw, rp0, rnp, rids = [], [], [], []
        for i in range(M):
            for ri in range(nr[i]):
                n = (n0[i], n1[i])[ri] if ri < 2 else 0
                rw.append(int((m1[i] >> ri) & 1) if ri < 2 else 0)
                rp0.append(p_first[i] + (0 if ri == 0 else n0[i]) if ri < 2 else p_first[i] + nparts[i])
                rnp.append(n)
                rids.append("%s%dr%d" % (prefix, base + i, ri) if ri < 2 else "%s%dx%d" % (prefix, base + i, ri - 2))
        self.rosters.append(winner=np.array(rw, dtype=np.int8), p0=np.array(rp0, dtype=np.int64),
                            np_=np.array(rnp, dtype=np.int32))
        self.r_ids.extend(rids)
        rows = self.matches.append(mode=np.where(mode < len(MODES), mode, UNSUPPORTED).astype(np.int16),
                                   created=(base + np.arange(M)).astype(np.float64), quality=np.full(M, NAN),
                                   r0=r_first, nr=nr.astype(np.int32))
        for a, r, md in zip(mids, rows, mode):
            self.m_index[a] = int(r)
        self.m_ids.extend(mids)
        self.m_mode_name.extend(MODES[x] if x < len(MODES) else "private" for x in mode)
        return mids

    def add_asset(self, match_api_id: str, url: str) -> None:
        self.assets_by_match.setdefault(match_api_id, []).append(url)

    def session(self) -> "ColumnarSession":
        return ColumnarSession(self)

    def close(self) -> None:
        pass

    # ------------------------------------------------------------- reads (tests)
    def player(self, api_id: str) -> Player:
        r = self.pl_index[api_id]
        kw = {c: _opt(v) for c, v in zip(PLAYER_COLS, self.players.rating[r])}
        rr, rb, tier = (_opt(v) for v in self.players.attr[r])
        return Player(api_id, None if tier is None else int(tier), rr, rb, **kw)


class ColumnarSession:
    """Transaction over a ColumnarStore: batch (columnar) and object access."""

    def __init__(self, store: ColumnarStore):
        self.store = store
        self._batches: List[MatchBatch] = []
        self._objects: Dict[int, Tuple[int, Match]] = {}   # id(match) -> (row, match)
        self._players: Dict[int, Player] = {}              # identity map by player row
        self.closed = False

    # ------------------------------------------------------------- columnar
    def _rows(self, ids: Iterable[str]) -> np.ndarray:
        rows = self.store.match_rows(ids if isinstance(ids, list) else list(ids))
        rows = np.unique(rows[rows >= 0])
        if rows.size:  # ORDER BY created_at (ties: insertion order)
            rows = rows[np.argsort(self.store.matches.created[rows], kind="stable")]
        return rows

    def load_batch(self, ids: Iterable[str], chunksize: int = 100) -> MatchBatch:
        """The batch's columns in one native pass (csrc/batch_host.cpp batch_gather);
        ``_load_batch_numpy`` is the vectorised reference the tests compare with."""
        st = self.store
        rows = self._rows(ids)
        mt, rt, pt = st.matches, st.rosters, st.parts
        t = torch.from_numpy
        mode, nr, n, winner, afk, player, part = (x.numpy() for x in native().batch_gather(
            t(rows), t(mt.nr), t(mt.r0), t(mt.mode), t(rt.np_), t(rt.winner), t(rt.p0), t(pt.player), t(pt.afk)))
        extra: Dict[int, List[int]] = {}
        for i in np.nonzero(nr > 2)[0]:  # participants of rosters beyond the second
            r0 = int(mt.r0[rows[i]])
            extra[int(i)] = [p for r in range(r0 + 2, r0 + int(nr[i]))
                             for p in range(int(rt.p0[r]), int(rt.p0[r]) + int(rt.np_[r]))]
        b = MatchBatch(ids=list(map(st.m_ids.__getitem__, rows.tolist())), mode=mode, nrosters=nr, n=n, winner=winner,
                       afk=afk, player=player, part=part, rows=rows, extra_parts=extra,
                       key_bound=st.players.n)
        self._batches.append(b)
        return b

    def _load_batch_numpy(self, ids: Iterable[str], chunksize: int = 100) -> MatchBatch:
        st = self.store
        rows = self._rows(ids)
        M = len(rows)
        mt, rt, pt = st.matches, st.rosters, st.parts
        nr = mt.nr[rows].astype(np.int64)
        r0 = mt.r0[rows]
        n = np.zeros((M, 2), dtype=np.int64)
        winner = np.zeros((M, 2), dtype=bool)
        p0 = np.zeros((M, 2), dtype=np.int64)
        for ri in range(2):
            has = nr > ri
            rr = np.where(has, r0 + ri, 0)
            n[:, ri] = np.where(has, rt.np_[rr], 0)
            winner[:, ri] = has & (rt.winner[rr] == 1)
            p0[:, ri] = rt.p0[rr]
        K = int(max(1, n.max() if M else 1))
        pos = np.arange(K)
        part = np.where(pos[None, None, :] < n[:, :, None], p0[:, :, None] + pos[None, None, :], -1)
        player = np.where(part >= 0, pt.player[np.maximum(part, 0)], -1)
        afkv = np.where(part >= 0, pt.afk[np.maximum(part, 0)] == 1, False)
        afk = afk_mask(n, afkv[:, 0], afkv[:, 1])
        extra: Dict[int, List[int]] = {}
        for i in np.nonzero(nr > 2)[0]:  # participants of rosters beyond the second
            ps = []
            for ri in range(2, int(nr[i])):
                r = int(r0[i]) + ri
                ps += list(range(int(rt.p0[r]), int(rt.p0[r]) + int(rt.np_[r])))
            extra[int(i)] = ps
            if any(pt.afk[p] == 1 for p in ps):
                afk[i] |= 1 << 23
        b = MatchBatch(ids=[st.m_ids[r] for r in rows], mode=mt.mode[rows].astype(np.int64), nrosters=nr,
                       n=n, winner=winner, afk=afk, player=player, part=part, rows=rows,
                       extra_parts=extra)
        self._batches.append(b)
        return b

    def fetch_players(self, keys: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Stored (ratings [n,14], attributes [n,3]) of player rows (resident upload)."""
        return self.store.players.rating[keys], self.store.players.attr[keys]

    def stage_players(self, keys: torch.Tensor, out: torch.Tensor) -> None:
        """``fetch_players`` straight into resident upload rows [n, 36]
        (csrc/batch_host.cpp batch_stage_players)."""
        pl = self.store.players
        native().batch_stage_players(keys, torch.from_numpy(pl.rating), torch.from_numpy(pl.attr), out)

    def _write_batch(self, b: MatchBatch) -> None:
        """One native pass (csrc/batch_host.cpp batch_commit) for the first two
        rosters; rosters beyond the second and telemetry stats here."""
        st = self.store
        mt, pt = st.matches, st.parts
        stt = b.status
        if stt is None:
            return
        if b.fields is None:
            return self._write_batch_numpy(b)
        t = torch.from_numpy
        native().batch_commit(t(b.rows), t(stt), t(b.quality), t(b.part), t(b.fields), t(b.mode),
                              t(b.final_keys), t(b.final), t(b.final_tracks), t(mt.quality), t(pt.i_afk),
                              t(pt.ts), t(pt.i_rating), t(st.players.rating))
        for i, ps in b.extra_parts.items():
            if stt[i] in (RATED, AFK, INVALID):
                pt.i_afk[ps] = 0 if stt[i] == RATED else 1
        if b.stats is not None:
            sel = stats_mask(stt)[:, None, None] & (b.part >= 0)
            pt.stats[b.part[sel]] = b.stats[sel]

    def _write_batch_numpy(self, b: MatchBatch) -> None:
        st = self.store
        mt, pt = st.matches, st.parts
        stt = b.status
        rated = stt == RATED
        afkm = (stt == AFK) | (stt == INVALID)
        mt.quality[b.rows[rated]] = b.quality[rated]
        mt.quality[b.rows[afkm]] = 0.0
        # any_afk: every participant of AFK / invalid matches True, of rated ones False
        for mask, val in ((afkm, 1), (rated, 0)):
            p = b.part[mask]
            pt.i_afk[p[p >= 0]] = val
            for i in np.nonzero(mask)[0]:
                if int(i) in b.extra_parts:
                    pt.i_afk[b.extra_parts[int(i)]] = val
        sel = rated[:, None, None] & (b.part >= 0)
        p = b.part[sel]
        pt.ts[p, 0] = b.s_mu[sel]
        pt.ts[p, 1] = b.s_sig[sel]
        pt.ts[p, 2] = b.delta[sel]
        mode = np.broadcast_to(b.mode[:, None, None], b.part.shape)[sel]
        pt.i_rating[p, 2 * mode] = b.m_mu[sel]
        pt.i_rating[p, 2 * mode + 1] = b.m_sig[sel]
        if b.stats is not None:
            ss = stats_mask(stt)[:, None, None] & (b.part >= 0)
            pt.stats[b.part[ss]] = b.stats[ss]
        if b.final_keys is not None and len(b.final_keys):
            cur = st.players.rating[b.final_keys]
            cols = np.repeat(b.final_tracks, 2, axis=1)  # (mu, sigma) of each touched track
            cur[cols] = b.final[cols]
            st.players.rating[b.final_keys] = cur

    # ------------------------------------------------------------- objects
    def _player(self, row: int) -> Player:
        pl = self._players.get(row)
        if pl is None:
            st = self.store
            kw = {c: _opt(v) for c, v in zip(PLAYER_COLS, st.players.rating[row])}
            rr, rb, tier = (_opt(v) for v in st.players.attr[row])
            pl = Player(st.pl_ids[row], None if tier is None else int(tier), rr, rb, **kw)
            self._players[row] = pl
        return pl

    def load_matches(self, ids: Iterable[str], chunksize: int = 100) -> Iterator[Match]:
        st = self.store
        mt, rt, pt = st.matches, st.rosters, st.parts
        for row in self._rows(ids):
            row = int(row)
            rosters = []
            for ri in range(int(mt.nr[row])):
                r = int(mt.r0[row]) + ri
                parts = []
                for p in range(int(rt.p0[r]), int(rt.p0[r]) + int(rt.np_[r])):
                    items = ParticipantItems(st.i_ids[p])
                    items.any_afk = None if pt.i_afk[p] < 0 else bool(pt.i_afk[p])
                    for c, v in zip(ITEM_COLS, pt.i_rating[p]):
                        setattr(items, c, _opt(v))
                    afk = None if pt.afk[p] < 0 else int(pt.afk[p])
                    tier = _opt(pt.tier[p])
                    part = Participant(self._player(int(pt.player[p])), st.p_ids[p], went_afk=afk,
                                       skill_tier=None if tier is None else int(tier), items=items)
                    part.trueskill_mu, part.trueskill_sigma, part.trueskill_delta = (
                        _opt(x) for x in pt.ts[p])
                    parts.append(part)
                w = int(rt.winner[r])
                rosters.append(Roster(parts, winner=None if w < 0 else bool(w), api_id=st.r_ids[r]))
            m = Match(st.m_mode_name[row], rosters, api_id=st.m_ids[row], created_at=float(mt.created[row]))
            m.trueskill_quality = _opt(mt.quality[row])
            self._objects[id(m)] = (row, m)
            yield m

    def _write_objects(self) -> None:
        st = self.store
        mt, pt = st.matches, st.parts
        for row, m in self._objects.values():
            mt.quality[row] = _nan(m.trueskill_quality)
            for part in m.participants:
                p = st.p_index[part.api_id]
                pt.ts[p] = [_nan(part.trueskill_mu), _nan(part.trueskill_sigma), _nan(part.trueskill_delta)]
                it = part.participant_items[0]
                pt.i_afk[p] = -1 if it.any_afk is None else int(bool(it.any_afk))
                pt.i_rating[p] = [_nan(getattr(it, c)) for c in ITEM_COLS]
                for ps in part.participant_stats or []:
                    pt.stats[p] = [_nan(getattr(ps, c)) for c in STAT_COLUMNS]
        for row, pl in self._players.items():
            st.players.rating[row] = [_nan(getattr(pl, c)) for c in PLAYER_COLS]

    # ------------------------------------------------------------- transaction
    def savepoint(self, m: Match) -> tuple:
        from .store import _get_item, _get_part, _get_player
        return ([(_get_part(p), _get_item(p.participant_items[0])) for p in m.participants],
                m.trueskill_quality, [(p.player[0], _get_player(p.player[0])) for p in m.participants])

    def restore(self, m: Match, sp: tuple) -> None:
        from .store import ITEM_WRITE_COLS, PARTICIPANT_WRITE_COLS, PLAYER_RATING_COLS
        parts, q, players = sp
        m.trueskill_quality = q
        for p, (pv, iv) in zip(m.participants, parts):
            for c, v in zip(PARTICIPANT_WRITE_COLS, pv):
                setattr(p, c, v)
            for c, v in zip(ITEM_WRITE_COLS, iv):
                setattr(p.participant_items[0], c, v)
        for pl, vals in players:
            for c, v in zip(PLAYER_RATING_COLS, vals):
                setattr(pl, c, v)

    def commit(self) -> None:
        for b in self._batches:
            self._write_batch(b)
        self._write_objects()
        self._batches.clear()
        self._objects.clear()
        self._players.clear()
        self.store.commits += 1

    def rollback(self) -> None:
        self._batches.clear()
        self._objects.clear()
        self._players.clear()

    def assets(self, match_api_id: str):
        from .store import Asset
        return [Asset(u, match_api_id) for u in self.store.assets_by_match.get(match_api_id, ())]

    def participant_stats(self, participant_api_id: str):
        p = self.store.p_index.get(participant_api_id)
        if p is None or np.isnan(self.store.parts.stats[p]).all():
            return None
        return {c: _opt(v) for c, v in zip(STAT_COLUMNS, self.store.parts.stats[p])}

    def close(self) -> None:
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
