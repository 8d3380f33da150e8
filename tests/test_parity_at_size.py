"""Per-round parity at BASELINE.json's full sizes (north star: bit-exact per-round membership/checksum parity at
16-64k members).

* config 2 (4,096 members, 1 % kill/revive churn, 200 rounds), config 4 (16,384 members, 2-way partition, Heal
  at rounds 60 and 80, run to the reference's convergence criterion, test_utils.go:164-199) and config 5's burst
  pattern at 4,096 members (10 % Reincarnate every 20 rounds, 100 rounds) against committed
  oracle fixtures (tests/golden/make_size_fixtures.py): every round, the sha256 of the checksum vector and of the
  phase-S targets, the three canonical state digests (rows, dissemination buffers, timer tables) and the protocol
  counters must be equal.
* config 3 at 65,536 members, bench.py's exact workload (kill at round 10), all 100 rounds against a committed
  fixture of the OpenMP oracle, every round as above; unsharded and split over 8 observer-row shards.
* a self-only start at 16,384 members (full syncs and reverse full syncs at size) against its fixture.
* config 3 at 65,536 members through the suspect AND faulty waves (75 rounds, kill at round 2): beyond the fixture,
  parity is checked through size-independent properties every 5 rounds: each sampled observer's checksum equals
  Fingerprint32 of the reference's checksum string (memberlist.go:106-128) rebuilt on the host from the engine's
  own row, and the killed members go alive -> suspect -> faulty in every sampled live row on the reference's
  timeouts (suspect 5 s = 25 rounds, state_transitions.go:90-117).
* config 5's bursts at 65,536 members on one GPU: the same row-rebuilt checksum property, no capacity error.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import swimsim
from swimsim import workloads as W
from oracle_ffi import fingerprint32

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STATUS = ["alive", "suspect", "faulty", "leave"]


def sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a).astype(dt).tobytes()).hexdigest()


def load_fixture(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {name}: run tests/golden/make_size_fixtures.py")
    with open(path) as f:
        return json.load(f)


def seed_rows(eng, wl):
    """the workload's MakeChange seeding before round 0 (tests/golden/make_size_fixtures.py seed_rows)"""
    for o in range(wl.n):
        for m in wl.seed_members:
            if m != o:
                eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE)


def compare_with_fixture(wl, fx, shards=None, on_round=None, **kw):
    """every round of the fixture: checksum vector, phase-S targets, the three state digests and the counters.
    shards: the same run split over that many observer-row shards of this process (ShardedCluster, LocalPort)."""
    assert fx["n"] == wl.n and fx["workload"] == wl.name
    eng = swimsim.ShardedCluster(wl.n, shards, init=wl.init, **kw) if shards else swimsim.Cluster(wl.n, init=wl.init, **kw)
    try:
        seed_rows(eng, wl)
        for rec in fx["records"]:
            r = rec["round"]
            assert eng.round == r
            eng.step(1, wl.events_for(r))
            got = {"checksums_sha256": sha(eng.checksums(), "<u4"), "targets_sha256": sha(eng.last_targets(), "<i4"),
                   "digest": [f"{x:016x}" for x in eng.digest()], "counters": eng.counters()}
            for k, v in got.items():
                assert v == rec[k], f"round {r}: {k} differs: engine {v} oracle {rec[k]}"
            if rec["converged"]:
                assert eng.converged(), f"round {r}: the oracle converged, the engine does not"
            if on_round:
                on_round(eng, r)
        return eng.counters(), fx["records"][-1]
    finally:
        eng.close()


def test_config2_full_size_200_rounds_vs_oracle_fixture():
    wl = W.config2(n=4096, rounds=200)
    c, last = compare_with_fixture(wl, load_fixture("config2_n4096.json"))
    assert last["round"] == 199
    assert c["pingreqs"] > 0 and c["applied"] > 0 and c["timers_fired"] > 0


def test_config4_full_size_to_convergence_vs_oracle_fixture():
    wl = W.config4(n=16384, rounds=260)
    c, last = compare_with_fixture(wl, load_fixture("config4_n16384.json"))
    assert last["converged"], "the fixture ends at convergence"
    assert c["heal_attempts"] > 0 and c["timers_fired"] > 0


def test_config3_n65536_bench_workload_vs_oracle_fixture():
    """bench.py's own workload at its own size, every round against the OpenMP oracle (north star: bit-exact
    per-round parity at 16-64k members): 65,536 members, 655 killed at round 10, all of config 3's 100 rounds
    (steady state, the kill, the suspect wave, the whole faulty wave from r = 35 on: state_transitions.go:90-117)."""
    fx = load_fixture("config3_n65536.json")
    wl = W.config3(n=65536, rounds=fx["rounds"], kill_round=10)
    c, last = compare_with_fixture(wl, fx)
    assert last["round"] == 99
    assert c["suspect_decl"] > 0 and c["timers_fired"] > 0 and c["pingreqs"] > 0


def test_config3_n65536_eight_shards_vs_oracle_fixture():
    """The 8-way observer-row split the north star names, at full size on one GPU: ShardedCluster(65536, 8) (eight
    shards of 8,192 rows in this process, cross-shard messages by device copies: the exchange RCCL carries between
    GPUs, ping_sender.go:90), every round against the same oracle fixture. Each shard's message pool is sized
    explicitly (the automatic size takes a share of the HBM left, which the first shards would exhaust). Records
    the bytes each shard exchanged per round."""
    fx = load_fixture("config3_n65536.json")
    wl = W.config3(n=65536, rounds=fx["rounds"], kill_round=10)
    per_round = []
    last = [0] * 8

    def xbytes(eng, r):
        now = [s["exchanged_bytes"] for s in eng.shard_info()]
        per_round.append([a - b for a, b in zip(now, last)])
        last[:] = now

    c, rec = compare_with_fixture(wl, fx, shards=8, on_round=xbytes, message_pool_bytes=4 << 30)
    assert rec["round"] == 99 and c["timers_fired"] > 0
    peak = max(max(x) for x in per_round)
    print(f"exchanged bytes per shard per round: peak {peak}, round 20 {per_round[20]}, round 60 {per_round[60]}")
    assert all(x > 0 for x in per_round[20])


def test_config3_n65536_two_shards_reference_row_path_vs_oracle_fixture():
    """Two shards of 32,768 rows: each shard's wide checksum launches run the reference-row path (a shard's reference
    row, divergent columns and exception records over its own rows), every round against the oracle fixture. Dense
    snapshot slots and message pools are sized explicitly so that both shards fit one GPU."""
    fx = load_fixture("config3_n65536.json")
    wl = W.config3(n=65536, rounds=fx["rounds"], kill_round=10)
    launches = []

    def paths(eng, r):
        launches.append(sum(s.checksum_path_stats()["delta_launches"] for s in eng.shards))

    c, rec = compare_with_fixture(wl, fx, shards=2, on_round=paths, message_pool_bytes=16 << 30,
                                  tuning={"dense_slots": 8192})
    assert rec["round"] == 99 and c["timers_fired"] > 0
    assert launches[-1] > 0, "no launch took the reference-row path"


def test_selfstart_n16384_full_syncs_vs_oracle_fixture():
    """Full syncs and reverse full syncs at size (disseminator.go:156-181, 257-304): 16,384 nodes that start knowing
    only themselves and two seeded members, 40 rounds, every round against the oracle fixture."""
    wl = W.selfstart(n=16384, seeds=2, rounds=40)
    c, last = compare_with_fixture(wl, load_fixture("selfstart_n16384.json"))
    assert last["round"] == 39
    assert last["counters"]["full_syncs"] > 0 and last["counters"]["rfs_done"] > 0
    assert c["full_syncs"] > 0 and c["rfs_done"] > 0


def test_config5_bursts_n4096_vs_oracle_fixture():
    wl = W.config5(n=4096, rounds=100)
    c, last = compare_with_fixture(wl, load_fixture("config5_n4096.json"))
    assert last["round"] == 99 and c["applied"] > 0


def checksum_from_row(st, inc):
    parts = [f"{swimsim.address_of(int(m))}{STATUS[st[m]]}{int(inc[m])};" for m in np.nonzero(st < 4)[0]]
    return fingerprint32("".join(parts).encode())


def test_config3_full_size_through_the_faulty_wave():
    n, kill = 65536, 2
    wl = W.config3(n=n, rounds=75, kill_round=kill)
    killed = np.array(sorted({e[2] for e in wl.events}))
    samples = [o for o in (0, 1, 777, 4097, 20000, 32768, 50001, 65535) if o not in set(killed.tolist())]
    eng = swimsim.Cluster(n)
    suspect_done = faulty_done = None
    try:
        for r0 in range(0, wl.rounds, 5):
            eng.step(5, [e for e in wl.events if r0 <= e[0] < r0 + 5])
            r = r0 + 4                                   # last round stepped
            cs = eng.checksums()
            states = []
            for o in samples + killed[:1].tolist():
                st, inc = eng.row(o)
                assert checksum_from_row(st, inc) == int(cs[o]), f"observer {o} after round {r}"
                if o in samples:
                    states.append(st[killed])
            ks = np.stack(states)
            # before the first suspect timer can fire (25 rounds after the first declaration) nothing is faulty
            if r < kill + 25:
                assert not (ks == swimsim.FAULTY).any(), f"faulty before any suspect timer could fire (round {r})"
            assert ((ks == swimsim.ALIVE) | (ks == swimsim.SUSPECT) | (ks == swimsim.FAULTY)).all()
            if suspect_done is None and (ks != swimsim.ALIVE).all():
                suspect_done = r
            if faulty_done is None and (ks == swimsim.FAULTY).all():
                faulty_done = r
        c = eng.counters()
        live_rounds = n * kill + (n - len(killed)) * (wl.rounds - kill)
        assert c["pings"] == live_rounds
        assert c["suspect_decl"] > 0 and c["timers_fired"] > 0
        assert suspect_done is not None and suspect_done < kill + 25, f"suspect wave incomplete ({suspect_done})"
        assert faulty_done is not None, "faulty wave incomplete at the end of the run"
        # every live row: every killed member faulty at the end
        for o in range(0, n, 4093):
            if o in set(killed.tolist()):
                continue
            st, _ = eng.row(o)
            assert (st[killed] == swimsim.FAULTY).all(), f"observer {o}"
        print(f"config3 n={n}: suspect wave complete by round {suspect_done}, faulty wave by {faulty_done}")
    finally:
        eng.close()


def test_config5_bursts_at_65536_on_one_gpu():
    """BASELINE.json config 5's burst pattern (10 % of the members Reincarnate every 20 rounds) at 65,536 members,
    the largest cluster whose rows, message pool and snapshots fit one MI355X (DESIGN.md §2 memory budget). A
    buffer holds up to ~1/4 of the members, so every message carries thousands of changes (no per-message cap,
    SURVEY.md §0.2). Checked: no capacity error, row-rebuilt checksums on sampled observers, every burst member
    known alive at its new incarnation everywhere once the burst has spread."""
    n = 65536
    wl = W.config5(n=n, rounds=64, every=20)
    eng = swimsim.Cluster(n)
    try:
        mem = eng.memory()
        assert mem["row_words"] + mem["dissemination"] + mem["timers"] < 21.2 * n * n
        eng.step(wl.rounds, wl.events)
        cs = eng.checksums()
        for o in (0, 12345, 65535):
            st, inc = eng.row(o)
            assert checksum_from_row(st, inc) == int(cs[o]), f"observer {o}"
        burst = sorted({e[2] for e in wl.events if e[0] == 40})
        st, inc = eng.row(777)
        assert (st[burst] == swimsim.ALIVE).all()
        assert (inc[burst] == swimsim.T0_MS + 40 * 200).mean() > 0.99
        c = eng.counters()
        assert c["applied"] > 1.5 * len(burst) * (n - 1) and c["msg_changes"] > 0
        print(f"config5 n={n}: {c['msg_changes'] / (n * wl.rounds):.0f} changes per message, memory {mem}")
    finally:
        eng.close()
