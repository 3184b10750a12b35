"""Synthetic match source for the worker (BASELINE config 1; SURVEY K7 host side).

In production the worker's input is a broker queue of match api ids whose rows
some other service has already written (/root/reference/worker.py:92,176).
Here the same pair is produced from the counter-based generator (the C++ host
mirror of the device generator, ops/synth.py): ``populate`` writes players,
matches, rosters, participants, items and telemetry assets into a store, and
``publish`` enqueues the match ids with optional ``notify`` headers -- exactly
what the worker consumes.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

from ..ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from .broker import BasicProperties
from .objects import Match, matches_from_stream, players_from_roster


def synth_objects(num_matches: int, num_players: int, team_size: int = 3, seed: int = 1,
                  stream: Optional[StreamSpec] = None, roster: Optional[RosterSpec] = None,
                  base: int = 0, prefix: str = "m"):
    """(players, matches) object graphs of a synthetic stream."""
    rspec = roster or RosterSpec(num_players=num_players, seed=seed)
    sspec = stream or StreamSpec(team_size=team_size, seed=seed + 1)
    r = make_roster(rspec)
    rec = make_stream(sspec, num_matches, rspec.num_players, K=sspec.team_size, base=base)
    players = players_from_roster(r.state, r.attrs)
    matches = matches_from_stream(rec, sspec.team_size, players, base=base, prefix=prefix)
    return players, matches


def populate(store, num_matches: int, num_players: int, team_size: int = 3, seed: int = 1,
             stream: Optional[StreamSpec] = None, roster: Optional[RosterSpec] = None,
             assets_per_match: int = 1, base: int = 0, prefix: str = "m"):
    """Write a synthetic stream into ``store``; returns the matches (objects), or
    for a ColumnarStore their api ids (bulk columnar insert, no objects)."""
    if hasattr(store, "add_stream"):
        return _populate_columnar(store, num_matches, num_players, team_size, seed, stream, roster,
                                  assets_per_match, base, prefix)
    players, matches = synth_objects(num_matches, num_players, team_size, seed, stream, roster,
                                     base, prefix)
    store.add_players(players)
    store.add_matches(matches)
    urls = [(m.api_id, "https://telemetry.invalid/%s/%d.json" % (m.api_id, a))
            for m in matches for a in range(assets_per_match)]
    if hasattr(store, "add_assets"):
        store.add_assets(urls)
    else:
        for mid, u in urls:
            store.add_asset(mid, u)
    return matches


class _Id(str):
    """A match api id that also answers ``.api_id`` (columnar populate results)."""

    @property
    def api_id(self) -> str:
        return str(self)


def _populate_columnar(store, num_matches, num_players, team_size, seed, stream, roster,
                       assets_per_match, base, prefix):
    import numpy as np

    from .columnar import ATTR_COLS, PLAYER_COLS  # noqa: F401  (column order documented there)

    rspec = roster or RosterSpec(num_players=num_players, seed=seed)
    sspec = stream or StreamSpec(team_size=team_size, seed=seed + 1)
    r = make_roster(rspec)
    st, at = r.state.double().numpy(), r.attrs.double().numpy()
    P = rspec.num_players
    ratings = np.empty((P, 14))
    ratings[:, 0::2] = st[:, 0:28:4]
    ratings[:, 1::2] = np.where(np.isnan(st[:, 0:28:4]), np.nan, st[:, 2:28:4])
    ids = ["p%d" % p for p in range(P)]
    keys = np.array([store.pl_index.get(a, -1) for a in ids], dtype=np.int64)
    new = keys < 0
    if new.any():
        store.add_player_arrays([a for a, n in zip(ids, new) if n], ratings[new], at[new, :3])
    keys = np.array([store.pl_index[a] for a in ids], dtype=np.int64)
    K = sspec.team_size
    rec = make_stream(sspec, num_matches, P, K=K, base=base).numpy().astype(np.int64)
    S = 2 * K
    slots = rec[:, :S]
    rec[:, :S] = np.where(slots >= 0, keys[np.maximum(slots, 0)], -1)  # player index -> store key
    mids = store.add_stream(rec, K, ids, base=base, prefix=prefix)
    for m in mids:
        for a in range(assets_per_match):
            store.add_asset(m, "https://telemetry.invalid/%s/%d.json" % (m, a))
    return [_Id(m) for m in mids]


def publish(channel, queue: str, ids: Sequence[str], notify: Optional[str] = None) -> None:
    """Enqueue match ids the way the producer service does (one message per match)."""
    for mid in ids:
        headers = {"notify": notify} if notify else {}
        channel.basic_publish(exchange="", routing_key=queue, body=mid.encode("utf-8"),
                              properties=BasicProperties(headers=headers))
