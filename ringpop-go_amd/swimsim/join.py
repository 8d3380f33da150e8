"""Join and bootstrap of a member into a running cluster.

The reference's joiner (swim/node.go:380-415, swim/join_sender.go:117-486):
  1. ``memberlist.Reincarnate`` (memberlist.go:234-236): MakeAlive(self, now) records its own change.
  2. ``sendJoin`` asks up to ``joinSize`` (default 3, join_sender.go:51) members; each answers with
     ``handleJoin`` (join_handler.go:52-77): its ``MembershipAsChanges`` and its checksum. The
     coordinator does not add the joiner; the others learn of it from its gossip.
  3. ``memberlist.AddJoinList`` (memberlist.go:398-406) per response: ``Update`` (override rules,
     timers by status via handleChanges, node.go:424-447), then ``ClearChange`` of every applied change
     except the joiner's own, so only its Reincarnate change is gossiped.
  4. gossip starts (node.go:405): the joiner is live from the next round.

``join`` replays this on any cluster object with the engine's setup calls (``make_change``,
``clear_changes``, ``set_live``, ``round``, ``row``). On the engine every call is the C ABI, so the
merges, timers and maxP updates are the device's. The response bodies pass through the JSON wire
format (swimsim.wire), as they would cross TChannel.

Two simplifications, both exact for a fresh joiner (a new swim.Node knows only itself):
  * The joiner's own entries in the join lists are skipped. Its Reincarnate incarnation is "now",
    newer than any the coordinators hold, so those entries neither apply nor trigger a refute.
  * Step 1 runs after step 3. The member changes never involve the joiner's row entry, and clearing
    every change before the Reincarnate leaves exactly the reference's final buffer.
Coordinators are taken in the order given. Go's join fan-out answers in network order.
"""
from __future__ import annotations

from typing import Iterable, List

from . import UNKNOWN, address_of
from . import wire as W


def _round(c):
    r = c.round
    return r() if callable(r) else r


def now_ms(cluster) -> int:
    """the joiner's clock, nowInMillis at the current round (T0 + r * P)"""
    return cluster.t0_ms + _round(cluster) * cluster.period_ms


def join(cluster, joiner: int, coordinators: Iterable[int], app: str = "ringpop") -> dict:
    """Join member `joiner` through `coordinators`; returns {"applied", "responses", "incarnation"}.

    On a cluster with ``add_join_list`` (the engine) the joiner runs the reference's order: Reincarnate, then
    one AddJoinList device launch per joinResponse. Elsewhere (the oracle view) the merges are replayed one
    ``make_change`` at a time and the Reincarnate comes last (see the module docstring: both orders leave the
    same state for a fresh joiner)."""
    coordinators = [int(c) for c in coordinators]
    if not coordinators:
        raise ValueError("join needs at least one coordinator (join_sender.go: no hosts to join)")
    if joiner in coordinators:
        # join_handler.go:36-42: a node may not join itself
        raise ValueError(f"member {joiner} tried to join the cluster by joining itself")
    device = hasattr(cluster, "add_join_list")
    applied = 0
    inc = now_ms(cluster)
    if device:
        cluster.make_change(joiner, joiner, inc, 0)     # Reincarnate: MakeAlive(self, now)
    req = W.JoinRequest(app, address_of(joiner), now_ms(cluster), 1_000_000_000)
    for c in coordinators:
        body = W.join_response(cluster, c, W.JoinRequest.from_json(req.to_json()).app).to_json()
        resp = W.JoinResponse.from_json(body)
        if resp.app != app:
            raise ValueError(f"coordinator {c} belongs to app {resp.app!r}, not {app!r}")
        cols = W.changes_to_arrays(resp.membership or [], cluster.n)
        if device:
            applied += cluster.add_join_list(joiner, cols["member"], cols["status"], cols["incarnation"],
                                             cols["source"], cols["source_incarnation"])
            continue
        for m, st, ic in zip(cols["member"].tolist(), cols["status"].tolist(), cols["incarnation"].tolist()):
            if m == joiner or st == UNKNOWN:
                continue
            applied += int(cluster.make_change(joiner, m, ic, st) or 0)
    if not device:
        cluster.clear_changes(joiner)                   # AddJoinList: ClearChange of every applied change
        cluster.make_change(joiner, joiner, inc, 0)     # Reincarnate: MakeAlive(self, now)
    cluster.set_live(joiner, 1)
    return {"applied": applied, "responses": len(coordinators), "incarnation": inc}


def bootstrap_order(n: int, seed_member: int = 0) -> List[int]:
    """members in join order after the seed (the discover provider's host list, in index order)"""
    return [m for m in range(n) if m != seed_member]


__all__ = ["join", "now_ms", "bootstrap_order"]
