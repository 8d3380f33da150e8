"""Parity of the MI355X engine (libswimsim.so, HIP path) with the CPU oracle.

Every round compares the per-observer checksums and the canonical digests of the member rows,
the dissemination buffers and the timer tables. It also compares the phase-S ping targets and
the protocol counters. Any divergence then gets a full-state diff to localize it. The bar is
bit-exact: everything here is integer/byte work.
"""
import numpy as np
import pytest

from oracle_ffi import OracleSim
import swimsim
from swimsim import workloads as W

pytestmark = pytest.mark.gpu


def make_pair(n, **kw):
    init = kw.pop("init", "converged")
    eng = swimsim.Cluster(n, init=init, **kw)
    okw = {k: v for k, v in kw.items() if k in ("t0_ms", "period_ms", "suspect_ms", "faulty_ms", "tombstone_ms",
                                                 "ping_request_size", "max_rfs_jobs", "p_factor", "seed")}
    ora = OracleSim(n, init=init, **okw)
    return eng, ora


def full_diff(eng, ora, n):
    msgs = []
    est, einc = eng.rows()
    ost, oinc = ora.rows()
    bad = np.argwhere((est != ost) | (einc != oinc))
    if len(bad):
        o, m = bad[0]
        msgs.append(f"row[{o}][{m}]: engine {est[o, m]},{einc[o, m]} oracle {ost[o, m]},{oinc[o, m]} ({len(bad)} diffs)")
    for o in range(n):
        if eng.changes(o) != ora.dis_entries(o):
            msgs.append(f"dissemination of {o}: engine {eng.changes(o)} oracle {ora.dis_entries(o)}")
            break
    for o in range(n):
        et = eng.timers(o)
        ot = ora.timer_entries(o)
        if et != ot:
            msgs.append(f"timers of {o}: engine {et} oracle {ot}")
            break
    ec, oc = eng.counters(), ora.counters()
    if ec != oc:
        msgs.append(f"counters: engine {ec} oracle {oc}")
    return "; ".join(msgs)


def run_parity(eng, ora, n, rounds, events=(), check_every=1, stop_when_converged=False):
    for r in range(rounds):
        evr = [e for e in events if e[0] == eng.round]
        eng.step(1, evr)
        ora.step(evr)
        if r % check_every and r != rounds - 1:
            continue
        et, ot = eng.last_targets(), ora.last_targets()
        assert (et == ot).all(), f"round {r}: targets differ at {np.nonzero(et != ot)[0][:5]}"
        ec, oc = eng.checksums(), ora.checksums()
        if not (ec == oc).all() or eng.digest() != ora.digest():
            pytest.fail(f"round {r}: divergence: {full_diff(eng, ora, n)}")
        if stop_when_converged and ora.converged():
            assert eng.converged()
            return r + 1
    assert eng.counters() == ora.counters()
    return rounds


def test_config1_kill_one_to_convergence():
    wl = W.config1()
    eng, ora = make_pair(wl.n)
    rounds = run_parity(eng, ora, wl.n, 120, wl.events)
    assert ora.counters()["timers_fired"] > 0
    st, _ = eng.row(0)
    assert st[5] == swimsim.FAULTY


def test_config2_churn_small():
    wl = W.config2(n=256, rounds=60)
    eng, ora = make_pair(wl.n)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    c = ora.counters()
    assert c["refutes"] + c["applied"] > 0 and c["pingreqs"] > 0


def test_config3_cascade_small():
    wl = W.config3(n=512, rounds=60, kill_round=5)
    eng, ora = make_pair(wl.n)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    assert ora.counters()["timers_fired"] > 0


def test_config4_partition_and_heal_small():
    wl = W.config4(n=64, rounds=110, split_until=40, heals=(40, 60))
    eng, ora = make_pair(wl.n)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    c = ora.counters()
    assert c["heal_attempts"] > 0 and c["full_syncs"] + c["rfs_done"] >= 0


def test_config5_bursts_small():
    wl = W.config5(n=300, rounds=45, every=15)
    eng, ora = make_pair(wl.n)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_tiny_clusters(n):
    eng, ora = make_pair(n)
    run_parity(eng, ora, n, 12, [(0, W.EV_KILL, n - 1, 0)] if n > 1 else [])


def test_zero_pingable_and_exhausted_iterator():
    # every other member dies: the survivors walk the whole permutation (memberlist_iter.go:50-72)
    n = 8
    eng, ora = make_pair(n)
    ev = [(0, W.EV_KILL, m, 0) for m in range(1, n)]
    run_parity(eng, ora, n, 40, ev)


def test_eviction_leave_reap_and_revive():
    n = 24
    kw = dict(faulty_ms=2000, tombstone_ms=1000)
    eng, ora = make_pair(n, **kw)
    ev = [(0, W.EV_KILL, 3, 0), (2, W.EV_LEAVE, 7, 0), (4, W.EV_KILL, 9, 0), (30, W.EV_REAP, 1, 0),
          (40, W.EV_REVIVE, 3, 0), (41, W.EV_REINCARNATE, 11, 0)]
    run_parity(eng, ora, n, 80, ev)
    assert ora.counters()["timers_fired"] > 0


def test_self_only_start_full_sync_and_merge():
    # nodes that only know themselves discover nothing by pinging; seed two rows by MakeChange
    n = 10
    eng, ora = make_pair(n, init="self")
    for o in range(n):
        for m in (0, 1):
            if m != o:
                assert eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE) == ora.make_change(o, m, swimsim.T0_MS, 0)
    run_parity(eng, ora, n, 40)


def test_partition_heal_reference_scenario():
    """heal_partition_test.go:36-77 on the round clock: A sees B faulty and vice versa."""
    n = 10
    eng, ora = make_pair(n, init="self")
    A, B = range(5), range(5, 10)
    for P in (A, B):
        for o in P:
            for m in P:
                eng.set_member(o, m, swimsim.ALIVE, swimsim.T0_MS)
                ora.set_member(o, m, 0, swimsim.T0_MS)
    for X, Y in ((A, B), (B, A)):
        for o in X:
            for m in Y:
                eng.make_change(o, m, swimsim.T0_MS, swimsim.FAULTY)
                ora.make_change(o, m, swimsim.T0_MS, 2)
            eng.clear_changes(o)
            ora.clear_changes(o)
    run_parity(eng, ora, n, 3)
    ev = [(eng.round, W.EV_HEAL, 0, 0), (eng.round + 30, W.EV_HEAL, 0, 0)]
    run_parity(eng, ora, n, 90, ev)
    st, _ = eng.row(7)
    assert (st[:10] == swimsim.ALIVE).all()


def test_api_views_match_oracle():
    n = 32
    eng, ora = make_pair(n)
    ev = [(0, W.EV_KILL, 4, 0)]
    run_parity(eng, ora, n, 10, ev)
    node = eng.node(0)
    assert node.GetChecksum() == ora.checksum(0)
    assert node.CountReachableMembers() == ora.count_reachable(0)
    assert node.memberlist.NumPingableMembers() == ora.num_pingable(0)
    assert node.disseminator.MaxP() == ora.maxp(0)
    assert node.disseminator.ChangesCount() == ora.changes_count(0)
    assert eng.iter_state(3) == ora.iter_state(3)
