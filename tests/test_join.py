"""Join and bootstrap (swimsim.join).

A cluster bootstraps from one seed member: every other member starts stopped and knowing only itself,
then joins through up to joinSize = 3 members already in (join_sender.go:51), taking their
joinResponse membership (join_handler.go:52-77, memberlist.go:398-406). CPU: the oracle alone
converges to a full alive membership. GPU: the engine and the oracle run the same joins and rounds
and match bit for bit each round (checksums, row/dissemination/timer digests, counters).
"""
import numpy as np
import pytest

import swimsim
from swimsim import join as J
from oracle_ffi import OracleSim


def _plan(n, every):
    """(round, joiner, coordinators): one member joins every `every` rounds through the first 3 joined"""
    out, joined = [], [0]
    for k, j in enumerate(J.bootstrap_order(n)):
        out.append((1 + k * every, j, joined[:3]))
        joined.append(j)
    return out


def _stop_all_but_seed(c, n):
    for m in range(1, n):
        c.set_live(m, 0)


def _run(clusters, n, rounds, every, check=None):
    plan = {r: (j, co) for r, j, co in _plan(n, every)}
    for _ in range(rounds):
        r = clusters[0].round
        if r in plan:
            j, co = plan[r]
            res = [J.join(c, j, co) for c in clusters]
            assert all(x == res[0] for x in res), f"join of {j}: {res}"
        for c in clusters:
            c.step(()) if isinstance(c, OracleSim) else c.step(1)
        if check:
            check(r)


def test_join_errors():
    ora = OracleSim(4, init="self")
    with pytest.raises(ValueError):
        J.join(ora, 1, [])
    with pytest.raises(ValueError):
        J.join(ora, 1, [1])


def test_bootstrap_converges_on_oracle():
    n, every = 12, 2
    ora = OracleSim(n, init="self")
    _stop_all_but_seed(ora, n)
    _run([ora], n, 1 + n * every + 60, every)
    st, inc = ora.rows()
    assert (st == swimsim.ALIVE).all(), "every member knows every other alive"
    assert len(set(ora.checksums().tolist())) == 1
    # each member's incarnation is its join round's clock (Reincarnate at join, memberlist.go:234-236)
    for r, j, _ in _plan(n, every):
        assert (inc[:, j] == ora.t0_ms + r * ora.period_ms).all()


def test_joiner_takes_coordinator_membership_without_gossiping_it():
    n = 8
    ora = OracleSim(n, init="self")
    _stop_all_but_seed(ora, n)
    J.join(ora, 1, [0])
    for _ in range(20):
        ora.step(())
    res = J.join(ora, 2, [0, 1])
    st, _ = ora.row(2)
    assert st[0] == st[1] == st[2] == swimsim.ALIVE and (st[3:] == swimsim.UNKNOWN).all()
    assert res["applied"] == 2                     # 0 and 1 from coordinator 0; coordinator 1 adds nothing new
    assert list(ora.dis_entries(2)) == [2]         # only its own Reincarnate change is disseminated


@pytest.mark.gpu
def test_gpu_bootstrap_parity_with_oracle():
    n, every = 48, 2
    eng = swimsim.Cluster(n, device=0, init="self")
    ora = OracleSim(n, init="self")
    _stop_all_but_seed(eng, n)
    _stop_all_but_seed(ora, n)

    def check(r):
        ec, oc = eng.checksums(), ora.checksums()
        assert (ec == oc).all(), f"round {r}: checksums differ at {np.nonzero(ec != oc)[0][:5]}"
        assert eng.digest() == ora.digest(), f"round {r}: state digests differ"
        assert eng.counters() == ora.counters(), f"round {r}: counters differ"

    _run([eng, ora], n, 1 + n * every + 40, every, check)
    st, _ = eng.rows()
    assert (st == swimsim.ALIVE).all()


@pytest.mark.gpu
@pytest.mark.parametrize("nshards", [2, 3])
def test_gpu_sharded_bootstrap_matches_single(nshards):
    """joins on observer-row shards (ShardedCluster routes each call to the joiner's owner shard)"""
    n, every = 40, 2
    one = swimsim.Cluster(n, device=0, init="self")
    sh = swimsim.ShardedCluster(n, nshards, init="self")
    _stop_all_but_seed(one, n)
    _stop_all_but_seed(sh, n)

    def check(r):
        assert (one.checksums() == sh.checksums()).all(), f"round {r}: checksums differ"
        assert one.digest() == sh.digest(), f"round {r}: state digests differ"

    _run([one, sh], n, 1 + n * every + 30, every, check)


def _join_list_case(n, seed):
    """a 3-row scenario: observer 1 knows a few members; the join list names most members with mixed statuses,
    unseen tombstones (Apply refuses to create them, memberlist.go:424-426), stale and newer incarnations, and
    observer 1 itself as suspect at its own incarnation (a refute, memberlist.go:337-354)"""
    rng = np.random.default_rng(seed)
    t0, per = swimsim.T0_MS, 200
    known = {m: (int(rng.integers(0, 3)), t0 + per * int(rng.integers(0, 4))) for m in range(0, n, 3)}
    known[1] = (swimsim.ALIVE, t0 + per * 5)
    lst = []
    for m in rng.permutation(n).tolist():
        if rng.random() < 0.15:
            continue
        st = int(rng.choice([0, 1, 2, 3, 4], p=[0.5, 0.15, 0.15, 0.05, 0.15]))
        lst.append((m, st, t0 + per * int(rng.integers(0, 6)), 0, t0 + per * 2))
    lst = [c for c in lst if c[0] != 1] + [(1, swimsim.SUSPECT, t0 + per * 5, 0, t0 + per * 2)]
    return known, lst


@pytest.mark.parametrize("seed", [1, 2])
def test_add_join_list_on_oracle_clears_all_but_own(seed):
    n = 64
    known, lst = _join_list_case(n, seed)
    ora = OracleSim(n, init="self")
    ora.set_round(6)
    for m, (st, inc) in known.items():
        ora.set_member(1, m, st, inc)
    ora.make_change(1, 1, swimsim.T0_MS + 6 * 200, swimsim.ALIVE)       # Reincarnate
    k = ora.add_join_list_changes(1, lst)
    assert k > 0
    assert list(ora.dis_entries(1)) == [1], "only the node's own change stays in the disseminator"
    st, _ = ora.row(1)
    unseen_tomb = [m for (m, s, *_r) in lst if s == swimsim.TOMBSTONE and m not in known]
    assert all(st[m] == swimsim.UNKNOWN for m in unseen_tomb)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_add_join_list_matches_oracle(seed):
    """swimsim_add_join_list (one device launch) against the oracle's AddJoinList restatement: the applied count,
    the row, the dissemination buffer and the timer table (per-row digests), the applied-change event"""
    n = 64
    known, lst = _join_list_case(n, seed)
    eng = swimsim.Cluster(n, device=0, init="self")
    ora = OracleSim(n, init="self")
    for c in (eng, ora):
        c.set_round(6)
        for m, (st, inc) in known.items():
            c.set_member(1, m, st, inc)
    eng.watch(1, True)
    ora.watch(1, True)
    for c in (eng, ora):
        c.make_change(1, 1, swimsim.T0_MS + 6 * 200, swimsim.ALIVE)
    cols = np.array(lst, dtype=np.int64)
    k_eng = eng.add_join_list(1, cols[:, 0], cols[:, 1], cols[:, 2], cols[:, 3], cols[:, 4])
    k_ora = ora.add_join_list_changes(1, lst)
    assert k_eng == k_ora > 0
    assert eng.digest() == ora.digest()
    assert (eng.checksums() == ora.checksums()).all()
    assert eng.changes(1).keys() == {1}
    ns = eng.node_stats(1)
    assert (ns["pingable"], ns["maxp"], ns["changes"]) == (ora.num_pingable(1), ora.maxp(1), 1)
    assert eng.applied_changes(1) == ora.drain_applied(1)          # MemberlistChangesAppliedEvent
