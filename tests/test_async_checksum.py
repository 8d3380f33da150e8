"""Phase C on the side stream: when few rows remain to hash after dedup, a round's
checksums are computed on a second HIP stream while the following rounds run. Rows whose checksum is
still pending refer to its side slot: a clean sender's C_o and a clean receiver's checksum in a
full-sync decision are read from that slot once the side stream has finished.

The overlap only happens inside one swimsim_step call of several rounds (a step returns with every
checksum current), so these tests step the engine several rounds at a time and compare with the
oracle at every chunk boundary, bit-exact. They also check that the side-stream path and the
synchronous path (swimsim_tuning.cs_async = 0) give identical states.
"""

import numpy as np
import pytest

import swimsim
from swimsim import workloads as W
from test_engine_parity import full_diff, make_pair
from test_sharded_parity import make_sharded

pytestmark = pytest.mark.gpu


def run_chunked(eng, ora, n, rounds, events=(), chunk=4):
    r = 0
    while r < rounds:
        k = min(chunk, rounds - r)
        r0 = eng.round
        eng.step(k, [e for e in events if r0 <= e[0] < r0 + k])
        for q in range(k):
            ora.step([e for e in events if e[0] == r0 + q])
        r += k
        ec, oc = eng.checksums(), ora.checksums()
        if not (ec == oc).all() or eng.digest() != ora.digest():
            pytest.fail(f"after round {r}: divergence: {full_diff(eng, ora, n)}")
    assert eng.counters() == ora.counters()


@pytest.mark.parametrize("chunk", [3, 8])
def test_chunked_config2_churn(chunk):
    wl = W.config2(n=256, rounds=48)
    eng, ora = make_pair(wl.n)
    run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk)


def test_chunked_config3_cascade():
    wl = W.config3(n=512, rounds=60, kill_round=5)
    eng, ora = make_pair(wl.n)
    run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk=10)
    assert ora.counters()["timers_fired"] > 0


def test_chunked_config4_partition_and_heal():
    wl = W.config4(n=64, rounds=110, split_until=40, heals=(40, 60))
    eng, ora = make_pair(wl.n)
    run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk=7)
    assert ora.counters()["heal_attempts"] > 0


def test_chunked_config5_bursts():
    wl = W.config5(n=300, rounds=45, every=15)
    eng, ora = make_pair(wl.n)
    run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk=9)


def test_chunked_self_only_full_syncs():
    """many full-sync decisions with clean receivers and senders whose checksums are pending"""
    n = 12
    eng, ora = make_pair(n, init="self")
    for o in range(n):
        for m in (0, 1):
            if m != o:
                assert eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE) == ora.make_change(o, m, swimsim.T0_MS, 0)
    run_chunked(eng, ora, n, 40, chunk=5)
    assert ora.counters()["full_syncs"] > 0


@pytest.mark.parametrize("shards", [2, 3])
def test_chunked_sharded_config2(shards):
    wl = W.config2(n=96, rounds=40)
    eng, ora = make_sharded(wl.n, shards)
    run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk=6)


def test_chunked_sharded_self_only():
    n = 10
    eng, ora = make_sharded(n, 3, init="self")
    for o in range(n):
        for m in (0, 1):
            if m != o:
                assert eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE) == ora.make_change(o, m, swimsim.T0_MS, 0)
    run_chunked(eng, ora, n, 40, chunk=5)
    assert ora.counters()["full_syncs"] > 0


def test_async_equals_sync_path():
    wl = W.config3(n=1024, rounds=50, kill_round=5)
    sync = swimsim.Cluster(wl.n, tuning={"cs_async": 0})
    asy = swimsim.Cluster(wl.n, tuning={"cs_async": 1})
    for r0 in range(0, wl.rounds, 10):
        ev = [e for e in wl.events if r0 <= e[0] < r0 + 10]
        sync.step(10, ev)
        asy.step(10, ev)
        assert (sync.checksums() == asy.checksums()).all(), f"checksums differ after round {r0 + 10}"
        assert sync.digest() == asy.digest(), f"state differs after round {r0 + 10}"
    assert sync.counters() == asy.counters()
    assert np.array_equal(sync.rows()[0], asy.rows()[0])


def test_side_stream_reference_row_path_vs_oracle():
    """The reference-row path on the side stream (its own buffer set, csr2): round-end launches of at least 1,024 rows
    (swimsim_tuning.fault_inject 256; 4,097 by default) hash their snapshots by k_csd_scan + k_csr3 on the side stream
    while the next rounds run. Bit-exact against the oracle at every chunk boundary of the cascade (memberlist.go:83-128),
    and the path did run (every wide-path launch here is a side launch: a 4,096-row main launch is narrow)."""
    wl = W.config3(n=4096, rounds=40, kill_round=5)
    eng, ora = make_pair(wl.n, tuning={"fault_inject": 256})
    run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk=5)
    st = eng.checksum_path_stats()
    print("side-stream reference-row path", st)
    assert st["delta_launches"] >= 1, st


def test_side_stream_reference_row_path_equals_narrow_kernel():
    """At 16,384 members, where the oracle is slow: the same cascade with the side set (fault_inject 256) and without
    it (128: side launches keep the narrow kernel) gives identical checksums, state digests and counters at every chunk
    boundary."""
    wl = W.config3(n=16384, rounds=30, kill_round=5)
    a = swimsim.Cluster(wl.n, tuning={"fault_inject": 256})
    b = swimsim.Cluster(wl.n, tuning={"fault_inject": 128})
    for r0 in range(0, wl.rounds, 5):
        ev = [e for e in wl.events if r0 <= e[0] < r0 + 5]
        a.step(5, ev)
        b.step(5, ev)
        bad = np.nonzero(a.checksums() != b.checksums())[0]
        assert len(bad) == 0, f"after round {r0 + 5}: {len(bad)} checksums differ, first {bad[:5]}"
        assert a.digest() == b.digest()
    assert a.counters() == b.counters()
    sa, sb = a.checksum_path_stats(), b.checksum_path_stats()
    print("side set", sa, "none", sb)
    assert sa["delta_launches"] > sb["delta_launches"], (sa, sb)


@pytest.mark.parametrize("tuning", [{"fault_inject": 1024}, {}])
def test_side_generations_vs_oracle(tuning):
    """Two generations of side-stream snapshot slots (default): phase C of a round snapshots into the half the round
    before did not use and does not wait for that round's side launch; a half's checksums reach cs[] when the half is
    reused or a full synchronisation retires it. Stepped 7 rounds per call (so up to three side launches overlap the
    main stream) through the cascade and churn, every chunk against the oracle; fault_inject 1024 keeps one generation."""
    for wl in (W.config3(n=1024, rounds=42, kill_round=5), W.config2(n=512, rounds=35)):
        eng, ora = make_pair(wl.n, tuning=tuning)
        run_chunked(eng, ora, wl.n, wl.rounds, wl.events, chunk=7)
