"""Reflected SQLAlchemy store: the reference's persistence layer.

The reference reflects whatever schema ``DATABASE_URI`` holds with
``automap_base`` and wires list-valued relationships on the ``api_id`` columns
by hand (/root/reference/worker.py:38-83), then loads each batch with one
ordered query, ``load_only`` column lists and chained ``selectinload``s,
``yield_per(CHUNKSIZE)`` (worker.py:176-191); here the same ordered query
eager-loads everything the rating touches instead (``load_matches``).  ``SqlAlchemyStore`` does the
same with SQLAlchemy 2.0 (the reference pins 1.2.0b1, whose string
``load_only("api_id")`` form 2.0 rejects -- SURVEY H7 -- so the column lists
are attribute objects here), for any URL a SQLAlchemy dialect + driver is
installed for: ``mysql+cymysql://`` in production (driver absent in this
image), ``sqlite:///file`` here.  The ORM objects carry the reference's column
names, so ``models.match_rater`` (ENGINE=python) and the resident-roster batch
rater (ENGINE=native) rate them unchanged.

Selected by ``STORE_BACKEND=sqlalchemy`` (with a sqlite URL), a
``sqlalchemy+<url>`` URI, or any URL scheme other than memory/columnar/sqlite
(runtime/store.open_store).

**Columnar batches (ENGINE=native).**  ``SqlAlchemySession.load_batch`` builds the
worker's ``MatchBatch`` (runtime/columnar.py) from four SQLAlchemy Core SELECTs per
batch -- matches ordered by ``created_at``, their rosters, their participants, the
participants' item rows -- with no ORM object at all; ``fetch_players`` reads the
stored ratings of the players the device roster has not seen; ``commit`` writes the
batch back as ``executemany`` UPDATEs keyed by primary key (match quality,
participant shared rating and delta, item ``any_afk`` + mode rating, the players'
final tracks) plus the ``participant_stats`` rows of DOTELEMETRY.  Only Core
constructs with bound parameters, so a MySQL URL takes the same statements.  Row
order follows what the reference's relationship loaders see (no ORDER BY on the
child tables: the database's order within a roster), so the columnar and the
object paths rate the same team lists (tests/test_worker.py).
"""
from __future__ import annotations

from typing import Dict, Iterable, Iterator, List, Optional

import numpy as np
from sqlalchemy import bindparam, create_engine, insert, select, text
from sqlalchemy.ext.automap import automap_base
from sqlalchemy.orm import relationship, selectinload, sessionmaker

from ..config import TRACK_COLUMNS
from .objects import STAT_COLUMNS
from .store import (ITEM_WRITE_COLS, PARTICIPANT_WRITE_COLS, PLAYER_RATING_COLS, SCHEMA, Asset,
                    _restore_match, _restore_player, _snap_match, _snap_player)

class SqlAlchemyStore:
    columnar_batches = True  # sessions build MatchBatch columns (load_batch / fetch_players)

    def __init__(self, uri: str, create_schema: bool = False):
        self.uri = uri
        kw = {"pool_recycle": 3600}
        if not uri.startswith("sqlite"):
            kw["pool_size"] = 1  # worker.py:44
        self.engine = create_engine(uri, **kw)
        if create_schema:
            with self.engine.begin() as c:
                for ddl in SCHEMA:
                    c.execute(text(ddl))
        Base = automap_base()
        Base.prepare(autoload_with=self.engine)
        C = Base.classes
        self.Asset, self.Match, self.Roster = C.asset, C.match, C.roster
        self.Participant, self.Player = C.participant, C.player
        self.ParticipantStats, self.ParticipantItems = C.participant_stats, C.participant_items
        # the reference's hand-wired, list-valued relationships (worker.py:52-82);
        # read-only here: the rater writes columns, never the links
        rel = lambda target, fk, join: relationship(target, foreign_keys=fk, primaryjoin=join, viewonly=True)
        self.Match.rosters = rel("roster", "roster.match_api_id", "match.api_id == roster.match_api_id")
        self.Match.participants = rel("participant", "participant.match_api_id",
                                      "match.api_id == participant.match_api_id")
        self.Roster.match = rel("match", "match.api_id", "match.api_id == roster.match_api_id")
        self.Roster.participants = rel("participant", "participant.roster_api_id",
                                       "roster.api_id == participant.roster_api_id")
        self.Participant.roster = rel("roster", "roster.api_id", "roster.api_id == participant.roster_api_id")
        self.Participant.match = rel("match", "match.api_id", "match.api_id == participant.match_api_id")
        self.Participant.player = rel("player", "player.api_id", "player.api_id == participant.player_api_id")
        self.Participant.participant_stats = rel(
            "participant_stats", "participant_stats.participant_api_id",
            "participant_stats.participant_api_id == participant.api_id")
        self.Participant.participant_items = rel(
            "participant_items", "participant_items.participant_api_id",
            "participant_items.participant_api_id == participant.api_id")
        Base.registry.configure()
        self.tables = Base.metadata.tables
        self.Session = sessionmaker(bind=self.engine, autoflush=False)
        self.commits = 0
        # integer keys of player api ids (columnar batches, device-resident roster rows)
        self.player_keys: Dict[str, int] = {}
        self.player_names: List[str] = []
        self._stmts: Dict[tuple, object] = {}

    def update_stmt(self, table: str, cols: tuple, key: str = "api_id"):
        """``UPDATE table SET cols WHERE key = :k_key`` with positional-free bound
        names (5v5_* columns start with a digit), cached per column set."""
        st = self._stmts.get((table, cols, key))
        if st is None:
            t = self.tables[table]
            st = (t.update().where(t.c[key] == bindparam("k_key"))
                  .values({c: bindparam("k%d" % i) for i, c in enumerate(cols)}))
            self._stmts[(table, cols, key)] = st
        return st

    # ------------------------------------------------------------- loading (synthetic data)
    def _insert(self, table: str, rows: List[dict]) -> None:
        if rows:
            with self.engine.begin() as c:
                c.execute(insert(self.tables[table]), rows)

    def add_players(self, players) -> None:
        cols = ("api_id", "skill_tier", "rank_points_ranked", "rank_points_blitz") + PLAYER_RATING_COLS
        self._insert("player", [{c: getattr(p, c) for c in cols} for p in players])

    def add_matches(self, matches) -> None:
        ms, rs, ps, its = [], [], [], []
        for m in matches:
            ms.append({"api_id": m.api_id, "game_mode": m.game_mode, "created_at": m.created_at,
                       "trueskill_quality": m.trueskill_quality})
            for r in m.rosters:
                rs.append({"api_id": r.api_id, "match_api_id": m.api_id,
                           "winner": None if r.winner is None else int(bool(r.winner))})
                for p in r.participants:
                    ps.append({"api_id": p.api_id, "match_api_id": m.api_id, "roster_api_id": r.api_id,
                               "player_api_id": p.player[0].api_id, "skill_tier": p.skill_tier,
                               "went_afk": p.went_afk, "trueskill_mu": p.trueskill_mu,
                               "trueskill_sigma": p.trueskill_sigma, "trueskill_delta": p.trueskill_delta})
                    it = p.participant_items[0]
                    row = {"api_id": it.api_id or p.api_id, "participant_api_id": p.api_id}
                    row.update({c: getattr(it, c) for c in ITEM_WRITE_COLS})
                    row["any_afk"] = None if row["any_afk"] is None else int(bool(row["any_afk"]))
                    its.append(row)
        for t, rows in (("match", ms), ("roster", rs), ("participant", ps), ("participant_items", its)):
            self._insert(t, rows)

    def add_assets(self, pairs) -> None:
        with self.engine.begin() as c:
            n = c.execute(text("SELECT COUNT(*) FROM asset")).scalar()
        self._insert("asset", [{"api_id": "a%d" % (n + i), "match_api_id": m, "url": u}
                               for i, (m, u) in enumerate(pairs)])

    def add_asset(self, match_api_id: str, url: str) -> None:
        self.add_assets([(match_api_id, url)])

    def session(self) -> "SqlAlchemySession":
        return SqlAlchemySession(self)

    def close(self) -> None:
        self.engine.dispose()


class SqlAlchemySession:
    """The worker's session interface over one ORM session."""

    def __init__(self, store: SqlAlchemyStore):
        self.store = store
        self.db = store.Session()
        self._snaps = {}  # id(match) -> snapshot for rollback of the in-memory objects
        self._players = {}
        self._batches: List = []  # columnar batches, written at commit
        self.closed = False

    # ------------------------------------------------------------- columnar batches
    def load_batch(self, ids: Iterable[str], chunksize: int = 100):
        """The batch as columns (runtime/columnar.MatchBatch) from Core SELECTs:
        no ORM objects, one statement per table and 500 keys."""
        from .columnar import MODE_INDEX, UNSUPPORTED, MatchBatch, afk_mask

        st = self.store
        t = st.tables
        Mt, Rt, Pt, It = t["match"], t["roster"], t["participant"], t["participant_items"]
        conn = self.db.connection()
        ids = list(set(ids))
        heads: List[tuple] = []
        for chunk in _chunks(ids, 500):
            heads += conn.execute(select(Mt.c.api_id, Mt.c.game_mode, Mt.c.created_at)
                                  .where(Mt.c.api_id.in_(chunk)).order_by(Mt.c.created_at.asc())).all()
        if len(ids) > 500:  # merge the chunks as ORDER BY would (NULL first, as MySQL / SQLite)
            heads.sort(key=lambda r: (r[2] is not None, r[2] if r[2] is not None else 0))
        mids = [h[0] for h in heads]
        pos = {m: i for i, m in enumerate(mids)}
        rosters: List[List[tuple]] = [[] for _ in mids]
        parts: Dict[str, List[tuple]] = {}
        for chunk in _chunks(mids, 500):
            for r in conn.execute(select(Rt.c.api_id, Rt.c.match_api_id, Rt.c.winner)
                                  .where(Rt.c.match_api_id.in_(chunk))):
                rosters[pos[r[1]]].append(r)
            for p in conn.execute(select(Pt.c.api_id, Pt.c.roster_api_id, Pt.c.player_api_id, Pt.c.went_afk)
                                  .where(Pt.c.match_api_id.in_(chunk))):
                parts.setdefault(p[1], []).append(p)
        pids = [p[0] for ps in parts.values() for p in ps]
        item_of: Dict[str, object] = {}
        for chunk in _chunks(pids, 500):
            for it in conn.execute(select(It.c.api_id, It.c.participant_api_id)
                                   .where(It.c.participant_api_id.in_(chunk))):
                item_of.setdefault(it[1], it[0])  # participant_items[0]
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
        keys, names = st.player_keys, st.player_names
        pnames: List[str] = []
        items: List[object] = []
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
                        items.append(item_of.get(p[0]))
                        afk23[i] |= p[3] == 1
                    continue
                winner[i, ri] = r[2] is not None and bool(r[2])
                for k, p in enumerate(ps):
                    k_ = keys.get(p[2])
                    if k_ is None:
                        k_ = keys[p[2]] = len(names)
                        names.append(p[2])
                    player[i, ri, k] = k_
                    part[i, ri, k] = len(pnames)
                    pnames.append(p[0])
                    items.append(item_of.get(p[0]))
                    afk[i, ri, k] = p[3] == 1
        mask = afk_mask(n, afk[:, 0], afk[:, 1]) | np.where(afk23, np.int64(1) << 23, 0)
        mode = np.array([MODE_INDEX.get(h[1], UNSUPPORTED) for h in heads], dtype=np.int64)
        b = MatchBatch(ids=mids, mode=mode, nrosters=nr, n=n, winner=winner, afk=mask, player=player,
                       part=part, player_names=pnames, extra_parts=extra)
        b.item_keys = items
        self._batches.append(b)
        return b

    def fetch_players(self, keys):
        """Stored (ratings [n, 14], attributes [n, 3]) of integer player keys."""
        Pl = self.store.tables["player"]
        names = [self.store.player_names[int(k)] for k in keys]
        cols = [Pl.c[c] for c in ("api_id", "rank_points_ranked", "rank_points_blitz", "skill_tier")
                + PLAYER_RATING_COLS]
        conn = self.db.connection()
        got = {}
        for chunk in _chunks(names, 500):
            for row in conn.execute(select(*cols).where(Pl.c.api_id.in_(chunk))):
                got[row[0]] = row[1:]
        att = np.full((len(names), 3), np.nan)
        rat = np.full((len(names), 14), np.nan)
        for i, a in enumerate(names):
            row = got.get(a)
            if row is not None:
                vals = np.array([np.nan if v is None else float(v) for v in row])
                att[i], rat[i] = vals[:3], vals[3:]
        return rat, att

    def _write_batch(self, b) -> None:
        """The batch's results as executemany UPDATEs keyed by primary key."""
        from .columnar import AFK, INVALID, RATED, stats_mask

        if b.status is None:
            return
        st = self.store
        conn = self.db.connection()
        stt = b.status
        rated = stt == RATED
        afkm = (stt == AFK) | (stt == INVALID)

        def run(table, cols, rows, key="api_id"):
            if rows:
                conn.execute(st.update_stmt(table, cols, key),
                             [dict(zip(["k%d" % i for i in range(len(cols))] + ["k_key"], r)) for r in rows])

        run("match", ("trueskill_quality",),
            [(float(b.quality[i]), b.ids[i]) for i in np.nonzero(rated)[0].tolist()] +
            [(0.0, b.ids[i]) for i in np.nonzero(afkm)[0].tolist()])
        items = b.item_keys
        flag = []  # any_afk: every participant of AFK / invalid matches (all rosters)
        for i in np.nonzero(afkm)[0].tolist():
            for p in b.part[i][b.part[i] >= 0].tolist() + b.extra_parts.get(i, []):
                flag.append((1, items[p]))
        for i in np.nonzero(rated)[0].tolist():  # rosters beyond the second of rated matches
            for p in b.extra_parts.get(i, []):
                flag.append((0, items[p]))
        run("participant_items", ("any_afk",), [f for f in flag if f[1] is not None])
        sel = rated[:, None, None] & (b.part >= 0)
        ps = b.part[sel].tolist()
        names = b.player_names
        run("participant", ("trueskill_mu", "trueskill_sigma", "trueskill_delta"),
            [(a, s_, d, names[p]) for a, s_, d, p in zip(b.s_mu[sel].tolist(), b.s_sig[sel].tolist(),
                                                            b.delta[sel].tolist(), ps)])
        mode = np.broadcast_to(b.mode[:, None, None], b.part.shape)[sel].tolist()
        by_mode: Dict[int, list] = {}
        for md, a, s_, p in zip(mode, b.m_mu[sel].tolist(), b.m_sig[sel].tolist(), ps):
            if items[p] is not None:  # any_afk = False and the mode rating at once
                by_mode.setdefault(md, []).append((0, a, s_, items[p]))
        for md, rows in by_mode.items():
            col = TRACK_COLUMNS[1 + md]
            run("participant_items", ("any_afk", col + "_mu", col + "_sigma"), rows)
        if b.stats is not None:
            self._write_stats(b, stats_mask(stt)[:, None, None] & (b.part >= 0))
        if b.final_keys is not None and len(b.final_keys):
            pn, f = st.player_names, b.final
            groups: Dict[tuple, list] = {}  # one UPDATE per set of touched tracks
            for u, k in enumerate(b.final_keys.tolist()):
                tracks = tuple(np.nonzero(b.final_tracks[u])[0].tolist())
                vals = []
                for tr in tracks:
                    mu, sg = f[u, 2 * tr], f[u, 2 * tr + 1]
                    vals += [None if mu != mu else float(mu), None if sg != sg else float(sg)]
                groups.setdefault(tracks, []).append(vals + [pn[int(k)]])
            for tracks, rows in groups.items():
                run("player", tuple(TRACK_COLUMNS[tr] + s for tr in tracks for s in ("_mu", "_sigma")), rows)

    def _write_stats(self, b, sel) -> None:
        """participant_stats rows (DOTELEMETRY): UPDATE the participants' existing
        rows, INSERT the others keyed by the participant api id -- no dialect
        specific upsert."""
        St = self.store.tables["participant_stats"]
        conn = self.db.connection()
        names = b.player_names
        vals = {names[p]: v for p, v in zip(b.part[sel].tolist(), b.stats[sel].tolist())}
        have = set()
        keys = list(vals)
        for chunk in _chunks(keys, 500):
            have.update(r[0] for r in conn.execute(select(St.c.participant_api_id)
                                                   .where(St.c.participant_api_id.in_(chunk))))
        upd = [list(vals[k]) + [k] for k in keys if k in have]
        if upd:
            conn.execute(self.store.update_stmt("participant_stats", STAT_COLUMNS, "participant_api_id"),
                         [dict(zip(["k%d" % i for i in range(len(STAT_COLUMNS))] + ["k_key"], r)) for r in upd])
        new = [dict(api_id=k, participant_api_id=k, **dict(zip(STAT_COLUMNS, vals[k]))) for k in keys if k not in have]
        if new:
            conn.execute(insert(St), new)

    def load_matches(self, ids: Iterable[str], chunksize: int = 100) -> Iterator:
        """The reference's batch query (worker.py:176-191), SQLAlchemy 2.0 spelling,
        with every relationship and column the rating touches loaded up front.

        The reference restricts the loaded columns (``load_only``) and leaves the
        participant items to lazy loading, so rating a match then issues one
        SELECT per item list, per deferred participant column group and per
        deferred player column (5v5 tracks, skill_tier): ~17 queries per 3v3
        match, measured 99 matches/s on sqlite:///file with ENGINE=native before
        this eager loading (profiles/r3/worker_sqla_native.json).  Same rows and
        values, six queries per chunk instead.  ENGINE=native takes ``load_batch``
        (columns, no objects) instead of this path."""
        s = self.store
        M, R, P = s.Match, s.Roster, s.Participant
        q = (select(M).where(M.api_id.in_(list(set(ids)))).order_by(M.created_at.asc())
             .options(selectinload(M.rosters).selectinload(R.participants)
                      .options(selectinload(P.player), selectinload(P.participant_items)),
                      selectinload(M.participants))
             .execution_options(yield_per=max(1, int(chunksize))))
        for m in self.db.scalars(q):
            self._snaps.setdefault(id(m), (m, _snap_match(m)))
            for p in m.participants:
                pl = p.player[0]
                self._players.setdefault(id(pl), (pl, _snap_player(pl)))
            yield m

    def savepoint(self, m) -> tuple:
        return (_snap_match(m), [(p.player[0], _snap_player(p.player[0])) for p in m.participants])

    def restore(self, m, sp: tuple) -> None:
        _restore_match(m, sp[0])
        for pl, snap in sp[1]:
            _restore_player(pl, snap)

    def commit(self) -> None:
        for b in self._batches:
            self._write_batch(b)
        self._batches.clear()
        self.db.commit()
        self.store.commits += 1
        self._snaps.clear()
        self._players.clear()

    def rollback(self) -> None:
        self._batches.clear()
        self.db.rollback()
        for m, snap in self._snaps.values():
            _restore_match(m, snap)
        for pl, snap in self._players.values():
            _restore_player(pl, snap)

    def assets(self, match_api_id: str) -> List[Asset]:
        A = self.store.Asset
        return [Asset(a.url, a.match_api_id) for a in
                self.db.scalars(select(A).where(A.match_api_id == match_api_id))]

    def participant_stats(self, participant_api_id: str):
        S = self.store.ParticipantStats
        row = self.db.scalars(select(S).where(S.participant_api_id == participant_api_id)).first()
        return None if row is None else {c: getattr(row, c) for c in STAT_COLUMNS}

    def close(self) -> None:
        self.db.close()
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def _chunks(seq, n: int):
    seq = list(seq)
    for i in range(0, len(seq), n):
        yield seq[i:i + n]


__all__ = ["SqlAlchemyStore", "SqlAlchemySession", "PARTICIPANT_WRITE_COLS"]
