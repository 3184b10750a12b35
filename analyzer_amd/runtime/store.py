"""State store of the worker: the reference's MySQL tables.

The reference reflects ``match, roster, participant, participant_items,
participant_stats, player, asset`` with SQLAlchemy automap and wires list-valued
relationships on the ``api_id`` foreign keys (/root/reference/worker.py:38-83).
That store is runtime/sqla.py (SQLAlchemy 2.0 is installed; the MySQL driver
the reference uses is not).  Every store sits behind one small session
interface:

    with store.session() as s:
        for match in s.load_matches(ids, chunksize):   # ORDER BY created_at ASC
            ...mutate objects...
        s.commit()       # or s.rollback()
        s.assets(match_api_id)

* ``MemoryStore`` keeps the object graph in process (tests, config 1, bench
  plumbing);
* ``SqliteStore`` (``DATABASE_URI=sqlite:///path``) stores the same tables and
  columns in SQLite through the standard library, with an identity map per
  session so one player that appears in several matches of a batch is ONE
  object -- exactly what the sequential rating semantics need
  (worker.py:191-192).

Both snapshot the writable fields of every loaded object so ``rollback()``
restores them (and ``restore(match)`` undoes a single quarantined match).
"""
from __future__ import annotations

import sqlite3
from dataclasses import dataclass
from operator import attrgetter
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

from ..config import TRACK_COLUMNS
from .objects import STAT_COLUMNS, Match, Participant, ParticipantItems, Player, Roster

PLAYER_RATING_COLS = tuple(c + s for c in TRACK_COLUMNS for s in ("_mu", "_sigma"))
ITEM_RATING_COLS = tuple(c + s for c in TRACK_COLUMNS[1:] for s in ("_mu", "_sigma"))
PARTICIPANT_WRITE_COLS = ("trueskill_mu", "trueskill_sigma", "trueskill_delta")
ITEM_WRITE_COLS = ("any_afk",) + ITEM_RATING_COLS


@dataclass
class Asset:
    url: str
    match_api_id: str


def _q(col: str) -> str:
    return '"%s"' % col  # 5v5_* columns start with a digit


class WriteConflict(RuntimeError):
    """A versioned player write found the row changed since the batch read it (another
    replica committed in between): the batch must be rolled back and rated again from
    fresh rows (runtime/worker.py).  The reference has no such check -- its replicas
    overwrite each other's player rows (/root/reference/worker.py:174-194)."""


SCHEMA = [
    # version: bumped by every rating write; replicas write with compare-and-set on it
    # (SqliteStore.versioned) -- a column the reference's schema does not have
    "CREATE TABLE IF NOT EXISTS player (api_id TEXT PRIMARY KEY, skill_tier INTEGER, "
    "rank_points_ranked REAL, rank_points_blitz REAL, %s, version INTEGER NOT NULL DEFAULT 0)"
    % ", ".join("%s REAL" % _q(c) for c in PLAYER_RATING_COLS),
    "CREATE TABLE IF NOT EXISTS match (api_id TEXT PRIMARY KEY, game_mode TEXT, "
    "created_at REAL, trueskill_quality REAL)",
    "CREATE INDEX IF NOT EXISTS match_created ON match(created_at)",
    "CREATE TABLE IF NOT EXISTS roster (api_id TEXT PRIMARY KEY, match_api_id TEXT, winner INTEGER)",
    "CREATE INDEX IF NOT EXISTS roster_match ON roster(match_api_id)",
    "CREATE TABLE IF NOT EXISTS participant (api_id TEXT PRIMARY KEY, match_api_id TEXT, "
    "roster_api_id TEXT, player_api_id TEXT, skill_tier INTEGER, went_afk INTEGER, "
    "trueskill_mu REAL, trueskill_sigma REAL, trueskill_delta REAL)",
    "CREATE INDEX IF NOT EXISTS participant_match ON participant(match_api_id)",
    "CREATE INDEX IF NOT EXISTS participant_roster ON participant(roster_api_id)",
    "CREATE TABLE IF NOT EXISTS participant_items (api_id TEXT PRIMARY KEY, "
    "participant_api_id TEXT, any_afk INTEGER, %s)" % ", ".join("%s REAL" % _q(c) for c in ITEM_RATING_COLS),
    "CREATE INDEX IF NOT EXISTS items_participant ON participant_items(participant_api_id)",
    "CREATE TABLE IF NOT EXISTS participant_stats (api_id TEXT PRIMARY KEY, "
    "participant_api_id TEXT, kills REAL, deaths REAL, assists REAL, damage REAL, "
    "gold REAL, farm REAL, healing REAL, events REAL)",
    # DOTELEMETRY commits look rows up and UPDATE them by participant (runtime/sqla.py
    # _write_stats); a reflected database needs the same index for the same reason
    "CREATE INDEX IF NOT EXISTS stats_participant ON participant_stats(participant_api_id)",
    "CREATE TABLE IF NOT EXISTS asset (api_id TEXT PRIMARY KEY, match_api_id TEXT, url TEXT)",
    "CREATE INDEX IF NOT EXISTS asset_match ON asset(match_api_id)",
]
# BATCH_LOG=true: every commit also records its matches in commit order (tests replay the
# log to show that no replica's update was lost)
BATCH_LOG_DDL = ("CREATE TABLE IF NOT EXISTS batch_log (seq INTEGER PRIMARY KEY AUTOINCREMENT, "
                 "replica TEXT, match_ids TEXT)")


def match_order(api_id: str, created_at) -> tuple:
    """Sort key of a batch: ``ORDER BY created_at ASC`` as the reference
    (/root/reference/worker.py:176), NULL first as MySQL / SQLite order it, and the
    api id breaking ties, so every store rates matches created at the same instant in
    one order (runtime/sqla.py issues the same ORDER BY created_at, api_id)."""
    return (created_at is not None, created_at if created_at is not None else 0.0, api_id)


# ---------------------------------------------------------------- snapshots
# attrgetter: one C call per object instead of a Python generator per column
_get_part = attrgetter(*PARTICIPANT_WRITE_COLS)
_get_item = attrgetter(*ITEM_WRITE_COLS)
_get_player = attrgetter(*PLAYER_RATING_COLS)


def _snap_match(m: Match) -> tuple:
    parts = m.participants
    return (m.trueskill_quality, [_get_part(p) for p in parts],
            [_get_item(p.participant_items[0]) for p in parts])


def _restore_match(m: Match, snap: tuple) -> None:
    q, parts, items = snap
    m.trueskill_quality = q
    for p, vals in zip(m.participants, parts):
        for c, v in zip(PARTICIPANT_WRITE_COLS, vals):
            setattr(p, c, v)
    for p, vals in zip(m.participants, items):
        for c, v in zip(ITEM_WRITE_COLS, vals):
            setattr(p.participant_items[0], c, v)


def _snap_player(pl: Player) -> tuple:
    return _get_player(pl)


def _restore_player(pl: Player, snap: tuple) -> None:
    for c, v in zip(PLAYER_RATING_COLS, snap):
        setattr(pl, c, v)


class _SessionBase:
    """Snapshot bookkeeping shared by both stores."""

    def __init__(self):
        self._match_snaps: Dict[int, Tuple[Match, tuple]] = {}
        self._player_snaps: Dict[int, Tuple[Player, tuple]] = {}
        self.closed = False

    def _track(self, m: Match) -> None:
        ms = self._match_snaps
        if id(m) not in ms:
            ms[id(m)] = (m, _snap_match(m))
        ps = self._player_snaps
        for p in m.participants:
            pl = p.player[0]
            if id(pl) not in ps:
                ps[id(pl)] = (pl, _get_player(pl))

    def savepoint(self, m: Match) -> tuple:
        """Snapshot of one match and its players (for per-match quarantine)."""
        return (_snap_match(m), [(p.player[0], _snap_player(p.player[0])) for p in m.participants])

    def restore(self, m: Match, sp: tuple) -> None:
        _restore_match(m, sp[0])
        for pl, snap in sp[1]:
            _restore_player(pl, snap)

    def rollback(self) -> None:
        for m, snap in self._match_snaps.values():
            _restore_match(m, snap)
        for pl, snap in self._player_snaps.values():
            _restore_player(pl, snap)

    def loaded_matches(self) -> List[Match]:
        return [m for m, _ in self._match_snaps.values()]

    def close(self) -> None:
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


# ---------------------------------------------------------------- in-memory
class MemorySession(_SessionBase):
    def __init__(self, store: "MemoryStore"):
        super().__init__()
        self.store = store

    def load_matches(self, ids: Iterable[str], chunksize: int = 100) -> Iterator[Match]:
        found = [self.store.matches[i] for i in set(ids) if i in self.store.matches]
        found.sort(key=lambda m: match_order(m.api_id, m.created_at))
        for m in found:
            self._track(m)
            yield m

    def commit(self) -> None:
        self.store.commits += 1
        self._match_snaps.clear()
        self._player_snaps.clear()

    def assets(self, match_api_id: str) -> List[Asset]:
        return list(self.store.assets.get(match_api_id, ()))

    def participant_stats(self, participant_api_id: str):
        for m in self.store.matches.values():
            for p in m.participants:
                if p.api_id == participant_api_id and p.participant_stats:
                    ps = p.participant_stats[0]
                    return {c: getattr(ps, c) for c in STAT_COLUMNS}
        return None


class MemoryStore:
    def __init__(self):
        self.matches: Dict[str, Match] = {}
        self.players: Dict[str, Player] = {}
        self.assets: Dict[str, List[Asset]] = {}
        self.commits = 0

    def add_players(self, players: Iterable[Player]) -> None:
        for p in players:
            self.players[p.api_id] = p

    def add_matches(self, matches: Iterable[Match]) -> None:
        for m in matches:
            self.matches[m.api_id] = m

    def add_asset(self, match_api_id: str, url: str) -> None:
        self.assets.setdefault(match_api_id, []).append(Asset(url, match_api_id))

    def session(self) -> MemorySession:
        return MemorySession(self)

    def close(self) -> None:
        pass


# ---------------------------------------------------------------- sqlite
class SqliteSession(_SessionBase):
    def __init__(self, store: "SqliteStore"):
        super().__init__()
        self.store = store
        self.conn = store.conn
        self._players: Dict[str, Player] = {}  # identity map
        self._batches: List = []
        self._versions: Dict[str, int] = {}    # api id -> version read (versioned stores)
        self._log_ids: List[str] = []          # matches of this transaction (BATCH_LOG)

    # ------------------------------------------------------------- columnar batches
    def load_batch(self, ids: Iterable[str], chunksize: int = 100):
        """The batch as columns (runtime/columnar.MatchBatch) from three SELECTs;
        player keys are the store's integer keys of their api ids."""
        import numpy as np

        from .columnar import MODE_INDEX, UNSUPPORTED, MatchBatch, afk_mask

        ids = list(set(ids))
        heads: List[tuple] = []
        for chunk in _chunks(ids, 500):
            heads += self.conn.execute(
                "SELECT api_id, game_mode, created_at FROM match WHERE api_id IN (%s)"
                % ", ".join("?" * len(chunk)), chunk).fetchall()
        heads.sort(key=lambda r: match_order(r[0], r[2]))
        mids = [h[0] for h in heads]
        pos = {m: i for i, m in enumerate(mids)}
        rosters: List[List[tuple]] = [[] for _ in mids]
        parts: Dict[str, List[tuple]] = {}
        for chunk in _chunks(mids, 500):
            ph = ", ".join("?" * len(chunk))
            for r in self.conn.execute("SELECT api_id, match_api_id, winner FROM roster WHERE "
                                       "match_api_id IN (%s) ORDER BY rowid" % ph, chunk):
                rosters[pos[r[1]]].append(r)
            for p in self.conn.execute(
                    "SELECT p.api_id, p.roster_api_id, p.player_api_id, p.went_afk, p.rowid, i.rowid "
                    "FROM participant p LEFT JOIN participant_items i ON i.participant_api_id = p.api_id "
                    "WHERE p.match_api_id IN (%s) ORDER BY p.rowid" % ph, chunk):
                parts.setdefault(p[1], []).append(p)
        M = len(mids)
        nr = np.array([len(r) for r in rosters], dtype=np.int64)
        n = np.zeros((M, 2), dtype=np.int64)
        for i, rs in enumerate(rosters):
            for ri in range(min(2, len(rs))):
                n[i, ri] = len(parts.get(rs[ri][0], ()))
        K = int(max(1, n.max() if M else 1))
        player = np.full((M, 2, K), -1, dtype=np.int64)
        part = np.full((M, 2, K), -1, dtype=np.int64)
        afk = np.zeros((M, 2, K), dtype=bool)
        winner = np.zeros((M, 2), dtype=bool)
        keys = self.store.player_keys
        pnames: List[str] = []
        prow: List[int] = []  # participant rowids (integer-key UPDATEs)
        irow: List[int] = []  # their participant_items rowids
        extra: Dict[int, List[int]] = {}
        afk23 = np.zeros(M, dtype=bool)
        for i, rs in enumerate(rosters):
            for ri, r in enumerate(rs):
                ps = parts.get(r[0], ())
                if ri >= 2:
                    ext = extra.setdefault(i, [])
                    for p in ps:
                        ext.append(len(pnames))
                        pnames.append(p[0])
                        prow.append(p[4])
                        irow.append(p[5])
                        afk23[i] |= p[3] == 1
                    continue
                winner[i, ri] = r[2] is not None and bool(r[2])
                for k, p in enumerate(ps):
                    k_ = keys.get(p[2])
                    if k_ is None:
                        k_ = keys[p[2]] = len(self.store.player_names)
                        self.store.player_names.append(p[2])
                    player[i, ri, k] = k_
                    part[i, ri, k] = len(pnames)
                    pnames.append(p[0])
                    prow.append(p[4])
                    irow.append(p[5])
                    afk[i, ri, k] = p[3] == 1
        mask = afk_mask(n, afk[:, 0], afk[:, 1]) | np.where(afk23, np.int64(1) << 23, 0)
        mode = np.array([MODE_INDEX.get(h[1], UNSUPPORTED) for h in heads], dtype=np.int64)
        b = MatchBatch(ids=mids, mode=mode, nrosters=nr, n=n, winner=winner, afk=mask, player=player,
                       part=part, player_names=pnames, extra_parts=extra)
        b.part_rowids = prow
        b.item_rowids = irow
        self._batches.append(b)
        return b

    def fetch_players(self, keys):
        """Stored (ratings [n,14], attributes [n,3]) of integer player keys."""
        import numpy as np

        pn = self.store.player_names
        names = [pn[k] for k in np.asarray(keys).tolist()]
        cols = ("api_id", "rowid", "rank_points_ranked", "rank_points_blitz", "skill_tier") + PLAYER_RATING_COLS
        if self.store.versioned:
            cols = cols + ("version",)
        rows: list = []
        for chunk in _chunks(names, 500):
            rows += self.conn.execute("SELECT %s FROM player WHERE api_id IN (%s)"
                                      % (", ".join(_q(c) for c in cols), ", ".join("?" * len(chunk))),
                                      chunk).fetchall()
        att = np.full((len(names), 3), np.nan)
        rat = np.full((len(names), 14), np.nan)
        if rows:
            # one numpy conversion (None -> NaN) instead of a Python float() per column
            where = {a: i for i, a in enumerate(names)}
            pos = np.fromiter((where[r[0]] for r in rows), dtype=np.int64, count=len(rows))
            if self.store.versioned:
                self._versions.update((r[0], r[-1]) for r in rows)
                rows = [r[:-1] for r in rows]
            vals = np.array([r[2:] for r in rows], dtype=np.float64)
            att[pos] = vals[:, :3]
            rat[pos] = vals[:, 3:]
            self.store.player_rowid.update((r[0], r[1]) for r in rows)
        return rat, att

    def _write_batch(self, b) -> None:
        import numpy as np

        from .columnar import AFK, INVALID, RATED

        if b.status is None:
            return
        c = self.conn
        st = b.status
        self._log_ids += list(b.ids)
        # the players first: with versioned rows a lost race (WriteConflict) shows before any
        # other row of the batch was written
        if b.final_keys is not None and len(b.final_keys):
            pn, prow_of = self.store.player_names, self.store.player_rowid
            f = np.asarray(b.final, dtype=np.float64)
            touched = np.asarray(b.final_tracks, dtype=bool)
            rowids = np.array([prow_of[pn[k]] for k in b.final_keys.tolist()], dtype=np.int64)
            # one UPDATE per set of touched tracks: players grouped by their track bitmask
            masks = (touched.astype(np.int64) << np.arange(touched.shape[1], dtype=np.int64)).sum(1)
            for m in np.unique(masks).tolist():
                if m == 0:
                    continue
                sel = masks == m
                tracks = [t for t in range(touched.shape[1]) if (m >> t) & 1]
                cols = np.array([[2 * t, 2 * t + 1] for t in tracks]).reshape(-1)
                vals = f[np.ix_(sel, cols)].astype(object)
                vals[np.isnan(f[np.ix_(sel, cols)])] = None  # NaN -> NULL
                rows = np.concatenate([vals, rowids[sel, None].astype(object)], axis=1).tolist()
                sets = ", ".join("%s=?, %s=?" % (_q(TRACK_COLUMNS[t] + "_mu"), _q(TRACK_COLUMNS[t] + "_sigma"))
                                 for t in tracks)
                if self.store.versioned:
                    # compare-and-set: only rows still at the version this batch read
                    ver = self._versions
                    vs = [ver.get(pn[k], 0) for k in np.asarray(b.final_keys)[sel].tolist()]
                    rows = [r + [v] for r, v in zip(rows, vs)]
                    cur = c.executemany("UPDATE player SET %s, version=version+1 WHERE rowid=? AND version=?"
                                        % sets, rows)
                    if cur.rowcount != len(rows):
                        raise WriteConflict("%d of %d player rows changed since this batch read them"
                                            % (len(rows) - max(cur.rowcount, 0), len(rows)))
                else:
                    c.executemany("UPDATE player SET %s WHERE rowid=?" % sets, rows)

        rated = st == RATED
        afkm = (st == AFK) | (st == INVALID)
        c.executemany("UPDATE match SET trueskill_quality=? WHERE api_id=?",
                      [(float(b.quality[i]), b.ids[i]) for i in np.nonzero(rated)[0]] +
                      [(0.0, b.ids[i]) for i in np.nonzero(afkm)[0]])
        names = b.player_names
        irow, rid = b.item_rowids, b.part_rowids
        sel = rated[:, None, None] & (b.part >= 0)
        # AFK / invalid: any_afk on every participant (incl. rosters beyond the second)
        flag = []
        for i in np.nonzero(afkm)[0]:
            for p in b.part[i][b.part[i] >= 0].tolist() + b.extra_parts.get(int(i), []):
                flag.append((1, irow[p]))
        c.executemany("UPDATE participant_items SET any_afk=? WHERE rowid=?", flag)
        extra = [(0, irow[p]) for i in np.nonzero(rated)[0] for p in b.extra_parts.get(int(i), [])]
        if extra:
            c.executemany("UPDATE participant_items SET any_afk=? WHERE rowid=?", extra)
        ps = b.part[sel].tolist()
        mu, sg, dl = b.s_mu[sel].tolist(), b.s_sig[sel].tolist(), b.delta[sel].tolist()
        c.executemany("UPDATE participant SET trueskill_mu=?, trueskill_sigma=?, trueskill_delta=? "
                      "WHERE rowid=?", [(a, s_, d, rid[p]) for a, s_, d, p in zip(mu, sg, dl, ps)])
        mode = np.broadcast_to(b.mode[:, None, None], b.part.shape)[sel].tolist()
        mm, ms = b.m_mu[sel].tolist(), b.m_sig[sel].tolist()
        by_mode: Dict[int, list] = {}
        for md, a, s_, p in zip(mode, mm, ms, ps):  # any_afk = False and the mode rating at once
            by_mode.setdefault(md, []).append((a, s_, irow[p]))
        for md, rows in by_mode.items():
            col = TRACK_COLUMNS[1 + md]
            c.executemany("UPDATE participant_items SET any_afk=0, %s=?, %s=? WHERE rowid=?"
                          % (_q(col + "_mu"), _q(col + "_sigma")), rows)
        if b.stats is not None:
            from .columnar import stats_mask

            ss = stats_mask(st)[:, None, None] & (b.part >= 0)
            st8 = b.stats[ss].tolist()
            c.executemany("INSERT OR REPLACE INTO participant_stats VALUES (?, ?, %s)"
                          % ", ".join("?" * len(STAT_COLUMNS)),
                          [[names[p], names[p]] + v for p, v in zip(b.part[ss].tolist(), st8)])
    def _load_players(self, api_ids: Sequence[str]) -> None:
        need = [a for a in set(api_ids) if a not in self._players]
        cols = ("api_id", "skill_tier", "rank_points_ranked", "rank_points_blitz") + PLAYER_RATING_COLS
        sel = cols + (("version",) if self.store.versioned else ())
        for chunk in _chunks(need, 500):
            rows = self.conn.execute(
                "SELECT %s FROM player WHERE api_id IN (%s)" % (", ".join(_q(c) for c in sel),
                                                                ", ".join("?" * len(chunk))), chunk)
            for row in rows:
                if self.store.versioned:
                    self._versions[row[0]] = row[-1]
                    row = row[:-1]
                kw = dict(zip(cols, row))
                api = kw.pop("api_id")
                tier = kw.pop("skill_tier")
                rr = kw.pop("rank_points_ranked")
                rb = kw.pop("rank_points_blitz")
                self._players[api] = Player(api, tier, rr, rb, **kw)

    def load_matches(self, ids: Iterable[str], chunksize: int = 100) -> Iterator[Match]:
        ids = list(set(ids))
        heads: List[tuple] = []
        for chunk in _chunks(ids, 500):
            heads += self.conn.execute(
                "SELECT api_id, game_mode, created_at, trueskill_quality FROM match "
                "WHERE api_id IN (%s)" % ", ".join("?" * len(chunk)), chunk).fetchall()
        heads.sort(key=lambda r: match_order(r[0], r[2]))
        # yield_per(chunksize): relationships are loaded one chunk of matches at a time
        for chunk in _chunks(heads, max(1, int(chunksize))):
            for m in self._build(chunk):
                self._track(m)
                yield m

    def _build(self, heads: Sequence[tuple]) -> List[Match]:
        mids = [h[0] for h in heads]
        ph = ", ".join("?" * len(mids))
        rosters: Dict[str, List[tuple]] = {}
        for r in self.conn.execute("SELECT api_id, match_api_id, winner FROM roster WHERE "
                                   "match_api_id IN (%s) ORDER BY rowid" % ph, mids):
            rosters.setdefault(r[1], []).append(r)
        parts = self.conn.execute(
            "SELECT api_id, match_api_id, roster_api_id, player_api_id, skill_tier, went_afk, "
            "trueskill_mu, trueskill_sigma, trueskill_delta FROM participant WHERE match_api_id "
            "IN (%s) ORDER BY rowid" % ph, mids).fetchall()
        self._load_players([p[3] for p in parts])
        pids = [p[0] for p in parts]
        items: Dict[str, ParticipantItems] = {}
        icols = ("api_id", "participant_api_id") + ITEM_WRITE_COLS
        for chunk in _chunks(pids, 500):
            for row in self.conn.execute(
                    "SELECT %s FROM participant_items WHERE participant_api_id IN (%s) ORDER BY rowid"
                    % (", ".join(_q(c) for c in icols), ", ".join("?" * len(chunk))), chunk):
                it = ParticipantItems(row[0])
                for c, v in zip(ITEM_WRITE_COLS, row[2:]):
                    setattr(it, c, bool(v) if c == "any_afk" and v is not None else v)
                items.setdefault(row[1], it)
        by_roster: Dict[str, List[Participant]] = {}
        by_match: Dict[str, List[Participant]] = {}
        for api, mid, rid, plid, tier, afk, mu, sig, dl in parts:
            pl = self._players.get(plid) or Player(plid)
            self._players.setdefault(plid, pl)
            p = Participant(pl, api, went_afk=afk, skill_tier=tier,
                            items=items.get(api) or ParticipantItems(api))
            p.trueskill_mu, p.trueskill_sigma, p.trueskill_delta = mu, sig, dl
            by_roster.setdefault(rid, []).append(p)
            by_match.setdefault(mid, []).append(p)
        out = []
        for api, mode, created, quality in heads:
            rs = [Roster(by_roster.get(r[0], []), winner=None if r[2] is None else bool(r[2]),
                         api_id=r[0]) for r in rosters.get(api, [])]
            m = Match(mode, rs, api_id=api, created_at=created)
            m.participants = by_match.get(api, [])
            m.trueskill_quality = quality
            out.append(m)
        return out

    def commit(self) -> None:
        c = self.conn
        for b in self._batches:
            self._write_batch(b)
        self._batches.clear()
        for m, _ in self._match_snaps.values():
            c.execute("UPDATE match SET trueskill_quality=? WHERE api_id=?", (m.trueskill_quality, m.api_id))
            for p in m.participants:
                for ps in getattr(p, "participant_stats", None) or []:
                    c.execute("INSERT OR REPLACE INTO participant_stats VALUES (?, ?, %s)"
                              % ", ".join("?" * len(STAT_COLUMNS)),
                              [ps.api_id or p.api_id, p.api_id] + [getattr(ps, x) for x in STAT_COLUMNS])
                c.execute("UPDATE participant SET trueskill_mu=?, trueskill_sigma=?, trueskill_delta=? "
                          "WHERE api_id=?", (p.trueskill_mu, p.trueskill_sigma, p.trueskill_delta, p.api_id))
                it = p.participant_items[0]
                vals = [getattr(it, col) for col in ITEM_WRITE_COLS]
                vals[0] = None if vals[0] is None else int(bool(vals[0]))
                c.execute("UPDATE participant_items SET %s WHERE participant_api_id=?"
                          % ", ".join("%s=?" % _q(col) for col in ITEM_WRITE_COLS), vals + [p.api_id])
        for pl, _ in self._player_snaps.values():
            sets = ", ".join("%s=?" % _q(col) for col in PLAYER_RATING_COLS)
            vals = [getattr(pl, col) for col in PLAYER_RATING_COLS] + [pl.api_id]
            if self.store.versioned:
                cur = c.execute("UPDATE player SET %s, version=version+1 WHERE api_id=? AND version=?" % sets,
                                vals + [self._versions.get(pl.api_id, 0)])
                if cur.rowcount != 1:
                    raise WriteConflict("player %s changed since this batch read it" % pl.api_id)
            else:
                c.execute("UPDATE player SET %s WHERE api_id=?" % sets, vals)
        if self.store.batch_log:
            ids = self._log_ids + [m.api_id for m, _ in self._match_snaps.values()]
            c.execute("INSERT INTO batch_log (replica, match_ids) VALUES (?, ?)",
                      (self.store.replica, ",".join(ids)))
        self._log_ids = []
        c.commit()
        self.store.commits += 1
        self._match_snaps.clear()
        self._player_snaps.clear()

    def lock(self) -> None:
        """Take the database's write lock now (BEGIN IMMEDIATE): a batch retried after a
        write conflict reads its players and commits under the lock, so it cannot lose
        again (runtime/worker.py ``process``)."""
        if not self.conn.in_transaction:
            self.conn.execute("BEGIN IMMEDIATE")

    def rollback(self) -> None:
        super().rollback()
        self._batches.clear()
        self._versions.clear()
        self._log_ids = []
        self.conn.rollback()

    def participant_stats(self, participant_api_id: str):
        row = self.conn.execute("SELECT %s FROM participant_stats WHERE participant_api_id=?"
                                % ", ".join(STAT_COLUMNS), (participant_api_id,)).fetchone()
        return None if row is None else dict(zip(STAT_COLUMNS, row))

    def assets(self, match_api_id: str) -> List[Asset]:
        return [Asset(u, m) for u, m in self.conn.execute(
            "SELECT url, match_api_id FROM asset WHERE match_api_id=? ORDER BY rowid", (match_api_id,))]


class SqliteStore:
    columnar_batches = True  # sessions build MatchBatch columns (load_batch / fetch_players)

    def __init__(self, path: str = ":memory:"):
        self.path = path
        # worker replicas share the file (runtime/replicas.py): a writer waits for the lock
        self.conn = sqlite3.connect(path, timeout=120.0)
        if path != ":memory:":
            # write-ahead log: a commit appends to the log instead of rewriting pages +
            # journal; NORMAL sync keeps every committed batch across a process crash
            self.conn.execute("PRAGMA journal_mode=WAL")
            self.conn.execute("PRAGMA synchronous=NORMAL")
        for ddl in SCHEMA:
            self.conn.execute(ddl)
        import os

        cols = {r[1] for r in self.conn.execute("PRAGMA table_info(player)")}
        cas = os.environ.get("PLAYER_CAS", "auto")
        if cas == "1" and "version" not in cols:  # an older file: add the column
            self.conn.execute("ALTER TABLE player ADD COLUMN version INTEGER NOT NULL DEFAULT 0")
            cols.add("version")
        # versioned player writes (compare-and-set, WriteConflict): on for a player table with
        # a version column unless PLAYER_CAS=0 (the reference's racing replicas)
        self.versioned = "version" in cols and cas != "0"
        self.batch_log = os.environ.get("BATCH_LOG") == "true"
        self.replica = os.environ.get("REPLICA") or ""
        if self.batch_log:
            self.conn.execute(BATCH_LOG_DDL)
        self.conn.commit()
        self.commits = 0
        # integer keys of player api ids (columnar batches, resident roster rows)
        self.player_keys: Dict[str, int] = {}
        self.player_names: List[str] = []
        self.player_rowid: Dict[str, int] = {}

    def session(self) -> SqliteSession:
        return SqliteSession(self)

    # ------------------------------------------------------------- loading
    def add_players(self, players: Iterable[Player]) -> None:
        cols = ("api_id", "skill_tier", "rank_points_ranked", "rank_points_blitz") + PLAYER_RATING_COLS
        self.conn.executemany(
            "INSERT OR REPLACE INTO player (%s) VALUES (%s)" % (", ".join(_q(c) for c in cols),
                                                               ", ".join("?" * len(cols))),
            [[getattr(p, c) for c in cols] for p in players])
        self.conn.commit()

    def add_matches(self, matches: Iterable[Match]) -> None:
        c = self.conn
        icols = ("api_id", "participant_api_id") + ITEM_WRITE_COLS
        for m in matches:
            c.execute("INSERT OR REPLACE INTO match VALUES (?, ?, ?, ?)",
                      (m.api_id, m.game_mode, m.created_at, m.trueskill_quality))
            for r in m.rosters:
                c.execute("INSERT OR REPLACE INTO roster VALUES (?, ?, ?)",
                          (r.api_id, m.api_id, None if r.winner is None else int(bool(r.winner))))
                for p in r.participants:
                    c.execute("INSERT OR REPLACE INTO participant VALUES (?, ?, ?, ?, ?, ?, ?, ?, ?)",
                              (p.api_id, m.api_id, r.api_id, p.player[0].api_id, p.skill_tier,
                               p.went_afk, p.trueskill_mu, p.trueskill_sigma, p.trueskill_delta))
                    it = p.participant_items[0]
                    vals = [it.api_id or p.api_id, p.api_id] + [getattr(it, col) for col in ITEM_WRITE_COLS]
                    vals[2] = None if vals[2] is None else int(bool(vals[2]))
                    c.execute("INSERT OR REPLACE INTO participant_items (%s) VALUES (%s)"
                              % (", ".join(_q(x) for x in icols), ", ".join("?" * len(icols))), vals)
        c.commit()

    def add_asset(self, match_api_id: str, url: str) -> None:
        self.add_assets([(match_api_id, url)])

    def add_assets(self, pairs) -> None:
        pairs = list(pairs)
        n = self.conn.execute("SELECT COUNT(*) FROM asset").fetchone()[0]
        self.conn.executemany("INSERT INTO asset VALUES (?, ?, ?)",
                              [("a%d" % (n + i), m, u) for i, (m, u) in enumerate(pairs)])
        self.conn.commit()

    def close(self) -> None:
        self.conn.close()


def _chunks(seq: Sequence, n: int):
    seq = list(seq)
    for i in range(0, len(seq), n):
        yield seq[i:i + n]


def open_store(uri: Optional[str], backend: Optional[str] = None):
    """Store for a ``DATABASE_URI``: None / ``memory://`` -> MemoryStore (object
    graph), ``columnar://`` -> ColumnarStore (numpy columns, the worker's fast
    native path), ``sqlite:///path`` (or ``sqlite://`` for an in-memory
    database) -> SqliteStore (stdlib sqlite3, columnar batches), and any other
    SQLAlchemy URL (``mysql+cymysql://...``), a ``sqlalchemy+<url>`` URI or
    ``STORE_BACKEND=sqlalchemy`` -> SqlAlchemyStore (automap reflection, the
    reference's relationships and batch query; runtime/sqla.py)."""
    import os

    backend = backend or os.environ.get("STORE_BACKEND") or ""
    if uri and uri.startswith("sqlalchemy+"):
        backend, uri = "sqlalchemy", uri[len("sqlalchemy+"):]
    if backend == "sqlalchemy" or (uri and not uri.startswith(("memory:", "columnar:", "sqlite:"))):
        from .sqla import SqlAlchemyStore
        # a sqlite file gets the reference's tables on first use; other servers must have them
        return SqlAlchemyStore(uri, create_schema=uri.startswith("sqlite"))
    if not uri or uri.startswith("memory:"):
        return MemoryStore()
    if uri.startswith("columnar:"):
        from .columnar import ColumnarStore
        return ColumnarStore()
    if uri.startswith("sqlite://"):
        path = uri[len("sqlite://"):]
        path = path[1:] if path.startswith("/") else path
        return SqliteStore(path or ":memory:")
    raise ValueError("unsupported DATABASE_URI %r" % uri)
