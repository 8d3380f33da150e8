"""Parity of a cluster whose observer rows are split over several shards (include/swimsim.h,
swimsim_group_create) with the CPU oracle, bit-exact per round.

The shards live in this process on one GPU and exchange their cross-shard traffic by device copies.
That is the same parcel protocol as the one-process-per-GPU RCCL transport, which differs only in
how the packed segments move. Every cross-shard path is exercised:
  - direct ping requests and responses (sparse and dense full-sync payloads);
  - ping-req relays through helpers on other shards;
  - reverse-full-sync sources pulled from other shards;
  - the collective heal (target membership and ping-with-changes across shards).
"""
import pytest

import swimsim
from swimsim import workloads as W
from oracle_ffi import OracleSim
from test_engine_parity import run_parity

pytestmark = pytest.mark.gpu


def make_sharded(n, shards, **kw):
    init = kw.pop("init", "converged")
    eng = swimsim.ShardedCluster(n, shards, init=init, **kw)
    okw = {k: v for k, v in kw.items() if k in ("t0_ms", "period_ms", "suspect_ms", "faulty_ms", "tombstone_ms",
                                                 "ping_request_size", "max_rfs_jobs", "p_factor", "seed")}
    return eng, OracleSim(n, init=init, **okw)


@pytest.mark.parametrize("shards", [2, 3])
def test_sharded_config1_to_convergence(shards):
    wl = W.config1()
    eng, ora = make_sharded(wl.n, shards)
    run_parity(eng, ora, wl.n, 120, wl.events)
    info = eng.shard_info()
    assert sum(i["hi"] - i["lo"] for i in info) == wl.n
    assert all(i["exchanges"] > 0 for i in info)


@pytest.mark.parametrize("shards", [2, 4])
def test_sharded_config2_churn(shards):
    wl = W.config2(n=256, rounds=50)
    eng, ora = make_sharded(wl.n, shards)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    assert ora.counters()["pingreqs"] > 0


def test_sharded_config3_cascade():
    wl = W.config3(n=512, rounds=50, kill_round=5)
    eng, ora = make_sharded(wl.n, 3)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    assert ora.counters()["timers_fired"] > 0


def test_sharded_config4_partition_and_heal():
    wl = W.config4(n=64, rounds=110, split_until=40, heals=(40, 60))
    eng, ora = make_sharded(wl.n, 2)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    assert ora.counters()["heal_attempts"] > 0


def test_sharded_config5_bursts():
    wl = W.config5(n=300, rounds=45, every=15)
    eng, ora = make_sharded(wl.n, 4)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)


def test_sharded_tiny_more_shards_than_rows_per_shard():
    n = 5
    eng, ora = make_sharded(n, 4)
    run_parity(eng, ora, n, 20, [(0, W.EV_KILL, 4, 0), (9, W.EV_REVIVE, 4, 0)])


def test_sharded_self_only_full_syncs():
    """dense full syncs and reverse full syncs between shards"""
    n = 10
    eng, ora = make_sharded(n, 3, init="self")
    for o in range(n):
        for m in (0, 1):
            if m != o:
                assert eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE) == ora.make_change(o, m, swimsim.T0_MS, 0)
    run_parity(eng, ora, n, 40)
    assert ora.counters()["full_syncs"] > 0 and ora.counters()["rfs_done"] > 0


def test_sharded_partition_heal_reference_scenario():
    """heal_partition_test.go:36-77 with the healing observer and its targets on different shards"""
    n = 10
    eng, ora = make_sharded(n, 2, init="self")
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
