"""The product's reference-row checksum path (csrc/swimsim_checksum_csr.hip: k_csd_scan + k_csr_ptable + k_csr_rec +
k_csr, and the production kernels for the rows it leaves) against the CPU oracle, bit for bit
(memberlist.go:83-128: every checksum is Fingerprint32 of the row's sorted member string).

The path is forced onto every phase-C launch of at least 1,024 rows (swimsim_tuning.cs_ref = 2, cs_async = 0 so that
every launch runs on the main stream) at sizes where the oracle runs every round: the cascade (rows a few records
apart), churn (incarnation bumps: longer and shorter records), a partition (rows half a membership apart: wide
shift ranges, workgroups whose window does not fit fall back), incarnation bursts and a self-only start (rows that
differ from the reference almost everywhere). At size, the path is compared with the engine's own checksums on real
cascade rows (swimsim_bench_checksum mode 5).
"""
import numpy as np
import pytest

from oracle_ffi import OracleSim
import swimsim
from swimsim import workloads as W

pytestmark = pytest.mark.gpu


def forced(n, **kw):
    return swimsim.Cluster(n, tuning={"cs_ref": 2, "cs_async": 0}, **kw)


def run_vs_oracle(wl, rounds, init="converged", seed_members=()):
    eng = forced(wl.n, init=init)
    ora = OracleSim(wl.n, init=init)
    for o in range(wl.n):
        for m in seed_members:
            if m != o:
                eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE)
                ora.make_change(o, m, swimsim.T0_MS, 0)
    for r in range(rounds):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        ec, oc = eng.checksums(), ora.checksums()
        bad = np.nonzero(ec != oc)[0]
        assert len(bad) == 0, f"round {r}: {len(bad)} checksums differ, first rows {bad[:5]}"
        assert eng.digest() == ora.digest(), f"round {r}: state digest differs"
    return eng


def test_cascade_n2048_every_round():
    wl = W.config3(n=2048, rounds=60, kill_round=5)
    eng = run_vs_oracle(wl, 60)
    st = eng.checksum_path_stats()
    print("cascade n2048", st)
    assert st["delta_launches"] >= 4, st


def test_churn_n2048_every_round():
    wl = W.config2(n=2048, rounds=40)
    eng = run_vs_oracle(wl, 40)
    st = eng.checksum_path_stats()
    print("churn n2048", st)
    assert st["delta_launches"] >= 5, st


def test_partition_n2048_every_round():
    wl = W.config4(n=2048, rounds=90)
    eng = run_vs_oracle(wl, 90)
    print("partition n2048", eng.checksum_path_stats())


def test_bursts_n2048_every_round():
    wl = W.config5(n=2048, rounds=45, every=20)
    eng = run_vs_oracle(wl, 45)
    print("bursts n2048", eng.checksum_path_stats())


def test_selfstart_n1024_every_round():
    wl = W.selfstart(n=1024, seeds=2, rounds=25)
    eng = run_vs_oracle(wl, 25, init="self", seed_members=wl.seed_members)
    print("selfstart n1024", eng.checksum_path_stats())


@pytest.mark.parametrize("n,rounds", [(4096, 18), (16384, 16)])
def test_mode5_on_real_cascade_rows(n, rounds):
    wl = W.config3(n=n, rounds=rounds + 1, kill_round=10)
    c = swimsim.Cluster(n)
    for r in range(rounds):
        c.step(1, wl.events_for(r))
    ref = c.checksums().copy()
    for rows in (1024, 3000, n):
        c.bench_checksum(rows, 5, reps=1)
        got = c.checksums()
        assert (got[:rows] == ref[:rows]).all(), f"{rows} rows: {(got[:rows] != ref[:rows]).sum()} differ"
    print(f"real rows n{n}", c.checksum_path_stats())


def test_stager_priority_schedule_on_real_cascade_rows():
    """swimsim_tuning.fault_inject = 16: k_csr3's stager waves at raised issue priority, a schedule in which one kind of
    chain wave (g/f or h) runs super steps ahead of the other. Each kind must count its own steps when a stager reuses
    a buffer: a count shared by both kinds let the leader's steps stand in for the laggard's, and the stager overwrote a
    window or code buffer the laggard was still reading (195 wrong rows of 65,536 at cascade round 18 in this schedule).
    The path's checksums must equal the production kernels' (swimsim_bench_checksum mode 0) on every row."""
    n = 32768
    wl = W.config3(n=n, rounds=21, kill_round=10)
    c = swimsim.Cluster(n, tuning={"fault_inject": 16})
    for r in range(20):
        c.step(1, wl.events_for(r))
        if r in (15, 17, 19):
            c.bench_checksum(n, 0, reps=1)
            ref = c.checksums().copy()
            for rep in range(2):
                c.bench_checksum(n, 5, reps=1)
                got = c.checksums()
                bad = np.nonzero(got != ref)[0]
                assert len(bad) == 0, f"round {r} rep {rep}: {len(bad)} rows differ, first {bad[:5]}"
    print("stager priority", c.checksum_path_stats())


def test_csr_alloc_failure_leaves_production_kernels_in_charge():
    """swimsim_tuning.fault_inject = 1: the reference-row path's buffers fail to allocate. The failure frees what was
    allocated and clears HIP's last error, so create and every step still succeed, on the production kernels."""
    wl = W.config3(n=2048, rounds=30, kill_round=5)
    eng = swimsim.Cluster(wl.n, tuning={"cs_ref": 2, "cs_async": 0, "fault_inject": 1})
    ora = OracleSim(wl.n)
    for r in range(30):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        assert (eng.checksums() == ora.checksums()).all(), f"round {r}"
    assert eng.checksum_path_stats()["delta_launches"] == 0


def test_csr_hash_hip_error_reaches_swimsim_step():
    """swimsim_tuning.fault_inject = 2: the first reference-row launch fails with SWIMSIM_EHIP. The error comes back from
    swimsim_step (HIP errors are mapped, never aborted on, and never swallowed), and the next handle
    works."""
    wl = W.config3(n=2048, rounds=30, kill_round=5)
    eng = swimsim.Cluster(wl.n, tuning={"cs_ref": 2, "cs_async": 0, "fault_inject": 2})
    with pytest.raises(swimsim.SwimsimError, match="EHIP"):
        for r in range(30):
            eng.step(1, wl.events_for(r))
    eng.close()
    run_vs_oracle(wl, 30)


def test_exception_overflow_slots_every_round():
    """swimsim_tuning.fault_inject = 4: 8 exception slots per stager wave, so waves spill into the window's unused tail
    (k_csr3's overflow slots) and, when that is full too, rows go to the production kernels. Bit-exact either way."""
    wl = W.config3(n=2048, rounds=40, kill_round=5)
    eng = swimsim.Cluster(wl.n, tuning={"cs_ref": 2, "cs_async": 0, "fault_inject": 4})
    ora = OracleSim(wl.n)
    for r in range(40):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        bad = np.nonzero(eng.checksums() != ora.checksums())[0]
        assert len(bad) == 0, f"round {r}: {len(bad)} checksums differ, first rows {bad[:5]}"
    st = eng.checksum_path_stats()
    print("overflow slots", st)
    assert st["delta_launches"] >= 4, st


def test_dedup_fingerprint_collision_groups():
    """swimsim_tuning.fault_inject = 8: dedup keys narrowed to 3 bits, so every fingerprint group holds unequal rows.
    k_fp_verify must hash every row that differs from its group head (memberlist.go:106-128: equal strings, equal
    checksums; only equality, never the fingerprint, decides a copy)."""
    for wl, rounds in ((W.config3(n=1024, rounds=30, kill_round=5), 30), (W.config2(n=1024, rounds=12), 12)):
        eng = swimsim.Cluster(wl.n, tuning={"fault_inject": 8})
        ora = OracleSim(wl.n)
        for r in range(rounds):
            ev = wl.events_for(r)
            eng.step(1, ev)
            ora.step(ev)
            bad = np.nonzero(eng.checksums() != ora.checksums())[0]
            assert len(bad) == 0, f"{wl.name} round {r}: {len(bad)} checksums differ"


def test_entry_cap_tail_rows_every_round():
    """swimsim_tuning.fault_inject = 32: at most 24 exception entries per row, so many rows end within the record
    stager's 4-entry prefetch of the cap (k_csr3 loads a record's first CSR_EREG entries with it; a clamp to cap - 4
    used to load the wrong entries for a record starting there). Rows past the cap go to the production kernels.
    Bit-exact either way, every round."""
    for wl, rounds in ((W.config3(n=2048, rounds=40, kill_round=5), 40), (W.config2(n=2048, rounds=25), 25)):
        eng = swimsim.Cluster(wl.n, tuning={"cs_ref": 2, "cs_async": 0, "fault_inject": 32})
        ora = OracleSim(wl.n)
        for r in range(rounds):
            ev = wl.events_for(r)
            eng.step(1, ev)
            ora.step(ev)
            bad = np.nonzero(eng.checksums() != ora.checksums())[0]
            assert len(bad) == 0, f"{wl.name} round {r}: {len(bad)} checksums differ, first rows {bad[:5]}"
        st = eng.checksum_path_stats()
        print("entry cap 24", wl.name, st)
        assert st["delta_launches"] >= 4, st


# (role bits of fault_inject 64: 1 g/f chains, 2 h chains, 4 record stagers, 8 window stagers)
JITTER_CASES = [(1, 11), (2, 12), (4, 13), (8, 14), (3, 15), (15, 16)]


@pytest.mark.parametrize("roles,seed", JITTER_CASES)
def test_perturbed_handover_on_real_cascade_rows(roles, seed):
    """swimsim_tuning.fault_inject = 64: seeded sleeps before k_csr3's hand-over waits and signals in the selected roles,
    so the g/f chains run ahead of the h chains (roles 2), the h chains ahead (1), a record stager (4) or a window stager
    (8) falls behind, or all of them drift (15). Every order must give the production kernels' checksums at 32,768 real
    cascade rows (swimsim_bench_checksum mode 5 against mode 0). A build with one done count shared by both kinds of
    chain wave (-DC3_T_SHAREDDONE, round 5's race) fails this test."""
    n = 32768
    wl = W.config3(n=n, rounds=21, kill_round=10)
    c = swimsim.Cluster(n, tuning={"fault_inject": 64 | (roles << 8) | (seed << 12)})
    for r in range(20):
        c.step(1, wl.events_for(r))
        if r in (15, 18):
            c.bench_checksum(n, 0, reps=1)
            ref = c.checksums().copy()
            c.bench_checksum(n, 5, reps=1)
            got = c.checksums()
            bad = np.nonzero(got != ref)[0]
            assert len(bad) == 0, f"roles {roles} round {r}: {len(bad)} rows differ, first {bad[:5]}"
    print("perturbed hand-over", roles, c.checksum_path_stats())


def test_colx_rebuild_after_raw_writes_every_round():
    """Raw row writes (swimsim_set_member; the reference's memberlist.Update applied without gossip) mark every column
    divergent, and the next step rebuilds DS::colx from the rows (k_colx_rebuild). The reference-row path (forced on
    every launch), the dedup comparison under 3-bit fingerprints (fault_inject 8) and the deferred decisions then compare
    rows over the rebuilt columns only: bit-exact against the oracle every round, with raw writes between rounds on a
    converged cluster and in the middle of the cascade."""
    wl = W.config3(n=2048, rounds=36, kill_round=5)
    eng = swimsim.Cluster(wl.n, tuning={"cs_ref": 2, "cs_async": 0, "fault_inject": 8})
    ora = OracleSim(wl.n)
    writes = {0: [(3, 7, 1, 1)], 12: [(100, 5, 0, 3), (101, 6, 2, 2)], 20: [(7, 9, 1, 4)]}
    for r in range(wl.rounds):
        for (o, m, st, k) in writes.get(r, ()):
            inc = swimsim.T0_MS + k * 200
            eng.set_member(o, m, st, inc)
            ora.set_member(o, m, st, inc)
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        bad = np.nonzero(eng.checksums() != ora.checksums())[0]
        assert len(bad) == 0, f"round {r}: {len(bad)} checksums differ, first rows {bad[:5]}"
        assert eng.digest() == ora.digest(), f"round {r}: state digest differs"


def test_side_stream_path_on_real_cascade_rows():
    """swimsim_bench_checksum mode 6: the reference-row path with the side-stream buffer set (csr2) on the side stream,
    as a round-end side launch runs it, over the first 8,192 and 12,288 rows of a 16,384-member cascade in the suspect
    wave: every checksum equals the engine's own (memberlist.go:83-128)."""
    n = 16384
    wl = W.config3(n=n, rounds=17, kill_round=10)
    c = swimsim.Cluster(n)
    for r in range(16):
        c.step(1, wl.events_for(r))
    ref = c.checksums().copy()
    for rows in (8192, 12288):
        ms = c.bench_checksum(rows, 6, reps=1)
        got = c.checksums()
        assert (got[:rows] == ref[:rows]).all(), f"{rows} rows: {(got[:rows] != ref[:rows]).sum()} differ"
        print(f"side-stream path, {rows} rows: {ms:.2f} ms")
