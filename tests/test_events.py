"""The upward coupling of the drop-in boundary: MemberlistChangesAppliedEvent (swim/events.go:56-61), which
memberlist.Update emits whenever it applied something (memberlist.go:366-384) and which Ringpop feeds its
hash ring from (ringpop.go:398-400,550-563), plus NodeInterface.ProtocolStats (stats.go:81-104).

A drain of a watched observer returns the last applied change of every member since the previous drain (the
per-Update events of the rounds in between, coalesced per member), the checksum at the previous drain
(OldChecksum), the current one (NewChecksum) and NumMembers. CPU tests pin the oracle's drain; GPU tests compare
the engine's drains with the oracle's every round and feed a device hash ring from them.

The per-Update stream (watch(o, "events"), swimsim_applied_events) does not coalesce: one event per Update that
applied something, in the node's Update order, so Ringpop's per-change statistics (ringpop.go:398-406) are the
reference's. CPU tests pin the oracle's stream against or_update's own return values; GPU tests compare the
engine's stream with the oracle's event by event every round (timers, full syncs, ping-reqs, heal, shards)."""
import numpy as np
import pytest

import swimsim
from swimsim import workloads as W
from oracle_ffi import OracleRing, OracleSim, UNKNOWN

WATCH = (0, 17, 100, 255)


def ring_ops(changes):
    """Ringpop.handleChanges (ringpop.go:550-563): alive/suspect add a server, faulty/leave/tombstone remove it"""
    add = [swimsim.address_of(m) for (m, st, *_r) in changes if st in (swimsim.ALIVE, swimsim.SUSPECT)]
    rem = [swimsim.address_of(m) for (m, st, *_r) in changes if st not in (swimsim.ALIVE, swimsim.SUSPECT)]
    return add, rem


def test_oracle_drain_is_the_coalesced_update_stream():
    wl = W.config2(n=128, rounds=30)
    ora = OracleSim(wl.n)
    for o in WATCH[:3]:
        ora.watch(o)
    prev = {o: ora.row(o) for o in WATCH[:3]}
    prev_cs = {o: ora.checksum(o) for o in WATCH[:3]}
    seen_changes = 0
    for r in range(wl.rounds):
        ora.step(wl.events_for(r))
        for o in WATCH[:3]:
            changes, old, new, nm = ora.drain_applied(o)
            st, inc = ora.row(o)
            assert old == prev_cs[o] and new == ora.checksum(o)
            assert nm == int(np.count_nonzero(st != UNKNOWN)) == ora.num_members(o)
            members = [c[0] for c in changes]
            assert members == sorted(set(members))                       # member order, one per member
            moved = set(np.nonzero((st != prev[o][0]) | (inc != prev[o][1]))[0].tolist())
            assert moved <= set(members)                                 # every state change was applied by Update
            for (m, cst, cinc, _s, _si) in changes:                      # the last applied change is the current state
                if st[m] != UNKNOWN:
                    assert (cst, cinc) == (int(st[m]), int(inc[m]))
            seen_changes += len(changes)
            prev[o], prev_cs[o] = (st, inc), new
        again, _, _, _ = ora.drain_applied(WATCH[0])
        assert again == []                                               # a drain clears the log
    assert seen_changes > 0


def _drains_match(eng, ora, observers, rings=None):
    for o in observers:
        e = eng.applied_changes(o)
        x = ora.drain_applied(o)
        assert e == x, f"observer {o}: engine {e[1:]} vs oracle {x[1:]}; {len(e[0])} vs {len(x[0])} changes"
        if rings is not None:
            g, orr = rings[o]
            add, rem = ring_ops(e[0])
            assert g.add_remove_servers(add, rem) == orr.add_remove_servers(add, rem)
            assert g.checksum() == orr.checksum() and g.server_count() == orr.server_count()


@pytest.mark.gpu
def test_gpu_applied_changes_match_oracle_and_feed_the_ring(gpu):
    """per round: the watched observers' drained changes, Old/NewChecksum and NumMembers equal the oracle's, and
    a device HashRing fed from them (Ringpop.handleChanges) equals the oracle ring fed from the oracle's"""
    from swimsim.ring import HashRing
    wl = W.config2(n=256, rounds=40)
    eng, ora = swimsim.Cluster(wl.n), OracleSim(wl.n)
    rings = {}
    for o in WATCH:
        eng.watch(o)
        ora.watch(o)
        g, orr = HashRing(100, device=0), OracleRing(100)
        everyone = [swimsim.address_of(m) for m in range(wl.n)]
        g.add_remove_servers(everyone)
        orr.add_remove_servers(everyone)
        rings[o] = (g, orr)
    total = 0
    for r in range(wl.rounds):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        for o in WATCH:
            total += len(ora.dis_entries(o))
        _drains_match(eng, ora, WATCH, rings)
    assert total > 0
    for g, _ in rings.values():
        g.close()


@pytest.mark.gpu
def test_gpu_applied_changes_coalesce_over_multi_round_steps(gpu):
    wl = W.config3(n=200, rounds=50, kill_round=2)
    eng, ora = swimsim.Cluster(wl.n), OracleSim(wl.n)
    for o in WATCH[:3]:
        eng.watch(o)
        ora.watch(o)
    for r0 in range(0, wl.rounds, 7):
        k = min(7, wl.rounds - r0)
        eng.step(k, [e for e in wl.events if r0 <= e[0] < r0 + k])
        for r in range(r0, r0 + k):
            ora.step(wl.events_for(r))
        _drains_match(eng, ora, WATCH[:3])


@pytest.mark.gpu
def test_gpu_applied_changes_sharded(gpu):
    wl = W.config2(n=192, rounds=25)
    eng, ora = swimsim.ShardedCluster(wl.n, 3), OracleSim(wl.n)
    watch = (0, 70, 150, 191)                                            # rows of all three shards
    for o in watch:
        eng.watch(o)
        ora.watch(o)
    for r in range(wl.rounds):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        _drains_match(eng, ora, watch)
    eng.close()


@pytest.mark.gpu
def test_gpu_register_listener_and_protocol_stats(gpu):
    wl = W.config1()
    eng = swimsim.Cluster(wl.n)
    got = []

    class Listener:                                                      # events.EventListener
        def HandleEvent(self, e):
            got.append(e)

    node = eng.node(3)
    node.RegisterListener(Listener())
    for r in range(40):
        eng.step(1, wl.events_for(r))
    assert got, "no MemberlistChangesAppliedEvent delivered"
    assert all(e.changes for e in got)
    assert got[-1].new_checksum == node.GetChecksum()
    assert got[-1].num_members == wl.n
    assert any(c.address == swimsim.address_of(5) and c.status == "faulty" for e in got for c in e.changes)
    for a, b in zip(got, got[1:]):
        assert b.old_checksum == a.new_checksum
    ps = node.ProtocolStats()
    t = ps["timing"]
    assert t["count"] == 40
    assert 0 < t["min_ns"] <= t["median_ns"] <= t["p95_ns"] <= t["max_ns"]
    assert abs(t["sum_ns"] - t["mean_ns"] * t["count"]) < 1e-3 * t["sum_ns"]
    assert ps["protocol_rate_ns"] == 200_000_000                         # max(2 x median, MinProtocolPeriod)
    assert ps["client_rate"] == 0 and ps["server_rate"] > 0


def _sorted_events(events):
    return [sorted(ev) for ev in events]


def test_oracle_event_stream_is_one_event_per_applying_update():
    n = 32
    ora = OracleSim(n)
    ora.watch(3, "events")
    ora.watch(3, "events")                                               # re-arming keeps the stream
    assert ora.drain_events(3)[0] == []
    t0 = ora.member(3, 7)[1]
    a1 = ora.update(3, [(7, 1, t0, 9, t0), (8, 1, t0, 9, t0)])           # two suspects: one Update
    a2 = ora.update(3, [(7, 1, t0, 9, t0)])                              # nothing new: no event
    a3 = ora.update(3, [(7, 2, t0, 10, t0)])                             # faulty: a second Update
    assert len(a1) == 2 and a2 == [] and len(a3) == 1
    events, old, new, nm = ora.drain_events(3)
    assert events == [a1, a3]
    assert nm == n and new == ora.checksum(3) and old != new
    assert ora.drain_events(3)[0] == []


def test_oracle_event_stream_refines_the_coalesced_drain():
    wl = W.config2(n=128, rounds=30)
    ora = OracleSim(wl.n)
    for o in WATCH[:3]:
        ora.watch(o, "events")
    nev = 0
    for r in range(wl.rounds):
        ora.step(wl.events_for(r))
        for o in WATCH[:3]:
            events, old, new, nm = ora.drain_events(o)
            coalesced, old2, new2, nm2 = ora.drain_applied(o)
            assert (old, new, nm) == (old2, new2, nm2)
            assert all(events)                                           # no empty event
            last = {}
            for ev in events:
                assert len({c[0] for c in ev}) == len(ev)                # one Update names a member once
                for c in ev:
                    last[c[0]] = c
            assert sorted(last.values()) == coalesced
            nev += len(events)
    assert nev > 0


def _events_match(eng, ora, observers):
    for o in observers:
        e = eng.applied_events(o)
        x = ora.drain_events(o)
        ee, xe = e[0], _sorted_events(x[0])
        assert len(ee) == len(xe), f"observer {o}: {len(ee)} events on the engine, {len(xe)} in the oracle"
        for k, (a, b) in enumerate(zip(ee, xe)):
            assert a == b, f"observer {o}, event {k}: engine {a[:4]}... vs oracle {b[:4]}..."
        assert e[1:] == x[1:], f"observer {o}: checksums / NumMembers {e[1:]} vs {x[1:]}"


def _run_events(eng, ora, wl, watch, per_call=1):
    for o in watch:
        eng.watch(o, "events")
        ora.watch(o, "events")
    total = 0
    for r0 in range(0, wl.rounds, per_call):
        k = min(per_call, wl.rounds - r0)
        eng.step(k, [e for e in wl.events if r0 <= e[0] < r0 + k])
        for r in range(r0, r0 + k):
            ora.step(wl.events_for(r))
        for o in watch:
            total += ora.changes_count(o)
        _events_match(eng, ora, watch)
    return total


@pytest.mark.gpu
def test_gpu_event_stream_matches_oracle_churn(gpu):
    wl = W.config2(n=256, rounds=40)
    eng, ora = swimsim.Cluster(wl.n), OracleSim(wl.n)
    assert _run_events(eng, ora, wl, WATCH) > 0
    c = ora.counters()
    assert c["pingreqs"] > 0 and c["timers_fired"] > 0


@pytest.mark.gpu
def test_gpu_event_stream_matches_oracle_timers_and_multi_round_steps(gpu):
    """the suspect and faulty waves: every fired timer is its own Update, in (deadline, member) order"""
    wl = W.config3(n=200, rounds=50, kill_round=2)
    eng, ora = swimsim.Cluster(wl.n), OracleSim(wl.n)
    _run_events(eng, ora, wl, WATCH[:3], per_call=7)
    assert ora.counters()["timers_fired"] > 0


@pytest.mark.gpu
def test_gpu_event_stream_matches_oracle_heal_and_full_syncs(gpu):
    wl = W.config4(n=128, rounds=70, split_until=30, heals=(30, 45))
    eng, ora = swimsim.Cluster(wl.n), OracleSim(wl.n)
    _run_events(eng, ora, wl, (0, 1, 64, 127))
    c = ora.counters()
    assert c["heal_attempts"] > 0


@pytest.mark.gpu
def test_gpu_event_stream_sharded(gpu):
    wl = W.config2(n=192, rounds=25)
    eng, ora = swimsim.ShardedCluster(wl.n, 3), OracleSim(wl.n)
    _run_events(eng, ora, wl, (0, 70, 150, 191))
    eng.close()
