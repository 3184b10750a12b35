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
from sqlalchemy import bindparam, create_engine, event, insert, select, text
from sqlalchemy.ext.automap import automap_base
from sqlalchemy.orm import relationship, selectinload, sessionmaker

from ..config import TRACK_COLUMNS
from .objects import STAT_COLUMNS
from .store import (ITEM_WRITE_COLS, PARTICIPANT_WRITE_COLS, PLAYER_RATING_COLS, SCHEMA, Asset, match_order,
                    _restore_match, _restore_player, _snap_match, _snap_player)

class SqlAlchemyStore:
    columnar_batches = True  # sessions build MatchBatch columns (load_batch / fetch_players)

    def __init__(self, uri: str, create_schema: bool = False):
        self.uri = uri
        kw = {"pool_recycle": 3600}
        if not uri.startswith("sqlite"):
            kw["pool_size"] = 1  # worker.py:44
        self.engine = create_engine(uri, **kw)
        if uri.startswith("sqlite") and ":memory:" not in uri and uri.rstrip("/") not in ("sqlite:", "sqlite:/"):
            # a sqlite FILE gets the stdlib store's settings (runtime/store.SqliteStore):
            # write-ahead log + NORMAL sync, every committed batch survives a process crash
            @event.listens_for(self.engine, "connect")
            def _sqlite_pragmas(dbapi_conn, _rec):
                c = dbapi_conn.cursor()
                c.execute("PRAGMA journal_mode=WAL")
                c.execute("PRAGMA synchronous=NORMAL")
                c.execute("PRAGMA cache_size=-262144")  # 256 MB of page cache (default 8 MB)
                c.execute("PRAGMA mmap_size=1073741824")
                c.close()
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

    def sql(self, key: tuple, build, names: List[str]):
        """A Core statement compiled once for this engine's dialect: (SQL text,
        parameter order, bound names).  The columnar path runs it on the DBAPI
        cursor, so the dialect's SQL and paramstyle come from SQLAlchemy without its
        per-row parameter and result processing (two thirds of a batch's store
        time through ``Connection.execute``)."""
        c = self._stmts.get(key)
        if c is None:
            comp = build().compile(dialect=self.engine.dialect)
            if self.engine.dialect.positional:
                at = {n: i for i, n in enumerate(names)}
                order = [at[n] for n in comp.positiontup]
                order = None if order == list(range(len(names))) else order
                c = (comp.string, "positional", order, names)
            else:
                c = (comp.string, "named", None, names)
            self._stmts[key] = c
        return c

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
    def _cursor(self):
        """A DBAPI cursor on the session's connection (the session's transaction)."""
        return self.db.connection().connection.dbapi_connection.cursor()

    def _select_in(self, cur, table: str, cols: tuple, key: str, values: List, order_by=None) -> List[tuple]:
        """``SELECT cols FROM table WHERE key IN (values)``, 500 bound values per
        statement (one compiled statement per chunk length)."""
        out: List[tuple] = []
        for chunk in _chunks(sorted(values), 500):  # key order: neighbouring index pages
            n = len(chunk)

            def build(n=n):
                t = self.store.tables[table]
                q = select(*[t.c[c] for c in cols]).where(t.c[key].in_([bindparam("i%d" % k) for k in range(n)]))
                return q.order_by(*[t.c[c].asc() for c in order_by]) if order_by else q
            c = self.store.sql(("in", table, cols, key, order_by, n), build, ["i%d" % k for k in range(n)])
            _execute(cur, c, [chunk])
            out += cur.fetchall()
        return out

    def load_batch(self, ids: Iterable[str], chunksize: int = 100):
        """The batch as columns (runtime/columnar.MatchBatch) from four SELECTs per
        500 keys: no ORM objects, no per-row SQLAlchemy processing."""
        from .columnar import MODE_INDEX, UNSUPPORTED, MatchBatch, afk_mask

        st = self.store
        cur = self._cursor()
        ids = list(set(ids))
        # ORDER BY created_at as the reference (worker.py:176), with api_id breaking ties so
        # that matches created at the same instant come out in one order on every path:
        # the chunked statements here, their merge below, and load_matches' single query
        heads = self._select_in(cur, "match", ("api_id", "game_mode", "created_at"), "api_id", ids,
                                order_by=("created_at", "api_id"))
        if len(ids) > 500:  # merge the chunks as ORDER BY would (NULL first, as MySQL / SQLite)
            heads.sort(key=lambda r: match_order(r[0], r[2]))
        mids = [h[0] for h in heads]
        pos = {m: i for i, m in enumerate(mids)}
        rosters: List[List[tuple]] = [[] for _ in mids]
        # no ORDER BY on the child tables: the database's order, as the reference's
        # relationship loaders see it (worker.py:176-191)
        for r in self._select_in(cur, "roster", ("api_id", "match_api_id", "winner"), "match_api_id", mids):
            rosters[pos[r[1]]].append(r)
        parts: Dict[str, List[tuple]] = {}
        for p in self._select_in(cur, "participant", ("api_id", "roster_api_id", "player_api_id", "went_afk"),
                                 "match_api_id", mids):
            parts.setdefault(p[1], []).append(p)
        pids = [p[0] for ps in parts.values() for p in ps]
        item_of: Dict[str, object] = {}
        for it in self._select_in(cur, "participant_items", ("api_id", "participant_api_id"),
                                  "participant_api_id", pids):
            item_of.setdefault(it[1], it[0])  # participant_items[0]
        cur.close()
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
        names = [self.store.player_names[int(k)] for k in keys]
        cols = ("api_id", "rank_points_ranked", "rank_points_blitz", "skill_tier") + PLAYER_RATING_COLS
        cur = self._cursor()
        got = {row[0]: row[1:] for row in self._select_in(cur, "player", cols, "api_id", names)}
        cur.close()
        nan = float("nan")
        vals = np.array([[nan if v is None else v for v in got.get(a, (None,) * 17)] for a in names],
                        dtype=np.float64).reshape(len(names), 17)
        return vals[:, 3:], vals[:, :3]

    def _update(self, cur, table: str, cols: tuple, rows: List[tuple], key: str = "api_id") -> None:
        """executemany ``UPDATE table SET cols WHERE key = ?`` of (values..., key) rows."""
        if not rows:
            return
        names = ["k%d" % i for i in range(len(cols))] + ["k_key"]

        def build():
            t = self.store.tables[table]
            return (t.update().where(t.c[key] == bindparam("k_key"))
                    .values({c: bindparam("k%d" % i) for i, c in enumerate(cols)}))
        # in key order: consecutive rows touch neighbouring index pages
        rows = sorted(rows, key=_last)
        _execute(cur, self.store.sql(("upd", table, cols, key), build, names), rows, many=True)

    def _write_batch(self, b) -> None:
        """The batch's results as executemany UPDATEs keyed by primary key."""
        from .columnar import AFK, INVALID, RATED, stats_mask

        if b.status is None:
            return
        st = self.store
        cur = self._cursor()
        stt = b.status
        rated = stt == RATED
        afkm = (stt == AFK) | (stt == INVALID)
        ri, ai = np.nonzero(rated)[0].tolist(), np.nonzero(afkm)[0].tolist()
        self._update(cur, "match", ("trueskill_quality",),
                     [(q, b.ids[i]) for i, q in zip(ri, b.quality[rated].tolist())] + [(0.0, b.ids[i]) for i in ai])
        items = b.item_keys
        flag = []  # any_afk: every participant of AFK / invalid matches (all rosters)
        for i in ai:
            for p in b.part[i][b.part[i] >= 0].tolist() + b.extra_parts.get(i, []):
                flag.append((1, items[p]))
        for i in ri:  # rosters beyond the second of rated matches
            for p in b.extra_parts.get(i, []):
                flag.append((0, items[p]))
        self._update(cur, "participant_items", ("any_afk",), [f for f in flag if f[1] is not None])
        sel = rated[:, None, None] & (b.part >= 0)
        ps = b.part[sel].tolist()
        names = b.player_names
        self._update(cur, "participant", ("trueskill_mu", "trueskill_sigma", "trueskill_delta"),
                     list(zip(b.s_mu[sel].tolist(), b.s_sig[sel].tolist(), b.delta[sel].tolist(),
                              [names[p] for p in ps])))
        mode = np.broadcast_to(b.mode[:, None, None], b.part.shape)[sel].tolist()
        by_mode: Dict[int, list] = {}
        for md, a, s_, p in zip(mode, b.m_mu[sel].tolist(), b.m_sig[sel].tolist(), ps):
            if items[p] is not None:  # any_afk = False and the mode rating at once
                by_mode.setdefault(md, []).append((0, a, s_, items[p]))
        for md, rows in by_mode.items():
            col = TRACK_COLUMNS[1 + md]
            self._update(cur, "participant_items", ("any_afk", col + "_mu", col + "_sigma"), rows)
        if b.stats is not None:
            self._write_stats(cur, b, stats_mask(stt)[:, None, None] & (b.part >= 0))
        if b.final_keys is not None and len(b.final_keys):
            pn = st.player_names
            ft = np.asarray(b.final_tracks, dtype=bool)
            code = ft.astype(np.int64).dot(np.int64(1) << np.arange(ft.shape[1], dtype=np.int64))
            for c in np.unique(code).tolist():  # one UPDATE per set of touched tracks
                u = np.nonzero(code == c)[0]
                tracks = [t for t in range(ft.shape[1]) if (c >> t) & 1]
                v = b.final[u][:, [x for t in tracks for x in (2 * t, 2 * t + 1)]]
                vo = v.astype(object)
                vo[np.isnan(v)] = None  # NULL
                self._update(cur, "player", tuple(TRACK_COLUMNS[t] + s for t in tracks for s in ("_mu", "_sigma")),
                             [tuple(r) + (pn[k],) for r, k in zip(vo.tolist(), b.final_keys[u].tolist())])
        cur.close()

    def _write_stats(self, cur, b, sel) -> None:
        """participant_stats rows (DOTELEMETRY): UPDATE the participants' existing
        rows, INSERT the others keyed by the participant api id -- no dialect
        specific upsert."""
        names = b.player_names
        vals = {names[p]: v for p, v in zip(b.part[sel].tolist(), b.stats[sel].tolist())}
        keys = list(vals)
        have = {r[0] for r in self._select_in(cur, "participant_stats", ("participant_api_id",),
                                              "participant_api_id", keys)}
        self._update(cur, "participant_stats", STAT_COLUMNS,
                     [tuple(vals[k]) + (k,) for k in keys if k in have], key="participant_api_id")
        new = [(k, k) + tuple(vals[k]) for k in keys if k not in have]
        if new:
            cols = ("api_id", "participant_api_id") + STAT_COLUMNS
            names_ = ["v%d" % i for i in range(len(cols))]

            def build():
                t = self.store.tables["participant_stats"]
                return insert(t).values({c: bindparam(n) for c, n in zip(cols, names_)})
            _execute(cur, self.store.sql(("ins", "participant_stats"), build, names_), new, many=True)

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
        q = (select(M).where(M.api_id.in_(list(set(ids)))).order_by(M.created_at.asc(), M.api_id.asc())
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


def _last(row):
    return row[-1]


def _execute(cur, compiled, rows: List[tuple], many: bool = False) -> None:
    """Run a ``SqlAlchemyStore.sql`` statement with tuple rows in bound-name order."""
    text_, style, order, names = compiled
    if style == "named":
        params = [dict(zip(names, r)) for r in rows]
    elif order is not None:
        params = [tuple(r[i] for i in order) for r in rows]
    else:
        params = rows if isinstance(rows, list) else list(rows)
    if many:
        cur.executemany(text_, params)
    else:
        cur.execute(text_, params[0])


def _chunks(seq, n: int):
    seq = list(seq)
    for i in range(0, len(seq), n):
        yield seq[i:i + n]


__all__ = ["SqlAlchemyStore", "SqlAlchemySession", "PARTICIPANT_WRITE_COLS"]
