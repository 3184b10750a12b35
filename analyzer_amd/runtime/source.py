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
             assets_per_match: int = 1, base: int = 0, prefix: str = "m") -> List[Match]:
    players, matches = synth_objects(num_matches, num_players, team_size, seed, stream, roster,
                                     base, prefix)
    store.add_players(players)
    store.add_matches(matches)
    for m in matches:
        for a in range(assets_per_match):
            store.add_asset(m.api_id, "https://telemetry.invalid/%s/%d.json" % (m.api_id, a))
    return matches


def publish(channel, queue: str, ids: Sequence[str], notify: Optional[str] = None) -> None:
    """Enqueue match ids the way the producer service does (one message per match)."""
    for mid in ids:
        headers = {"notify": notify} if notify else {}
        channel.basic_publish(exchange="", routing_key=queue, body=mid.encode("utf-8"),
                              properties=BasicProperties(headers=headers))
