"""BASELINE.json config 5 (large incarnation bursts) beyond its reduced-size parity case: the dense-snapshot
budget. A reincarnation burst dirties many rows at once, and lazy C_o (k_issue) would take one dense snapshot
per dirty sender. When the snapshot slots could not hold them, the engine hashes the dirty senders before issue
instead (bound_lazy_snapshots): exact either way. These tests force a small slot pool so that the
fallback runs, and compare every round with the oracle."""

import pytest

import swimsim
from swimsim import workloads as W
from test_engine_parity import make_pair, run_parity

pytestmark = pytest.mark.gpu


def _small_pool_pair(n, cap=64):
    return make_pair(n, tuning={"dense_slots": cap})


def test_config5_bursts_with_a_small_snapshot_pool():
    wl = W.config5(n=768, rounds=50, every=20)                 # 76 members reincarnate at r = 0, 20, 40
    eng, ora = _small_pool_pair(wl.n)
    mem = eng.memory()
    assert mem["dense_cap"] == 64
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    assert eng.memory()["lazy_fallbacks"] > 0
    c = ora.counters()
    assert c["applied"] > 0 and c["refutes"] >= 0


def test_config3_faulty_wave_with_a_small_snapshot_pool():
    # every row fires its suspect timers in the same rounds: all senders dirty at issue
    wl = W.config3(n=512, rounds=45, kill_round=3)
    eng, ora = _small_pool_pair(wl.n)
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)
    assert ora.counters()["timers_fired"] > 0
    assert eng.memory()["lazy_fallbacks"] > 0


def test_memory_budget_accounting():
    n = 4096
    eng = swimsim.Cluster(n)
    m = eng.memory()
    np_ = (n + 63) // 64 * 64
    assert m["row_words"] == n * np_ * 4
    assert m["dissemination"] >= n * np_ * 8 and m["timers"] >= n * np_ * 9
    assert m["total"] >= m["row_words"] + m["dissemination"] + m["timers"] + m["message_pool"] + m["dense_snapshots"]
    assert m["dense_cap"] >= 64


def test_config5_shard_allocates_on_one_mi355x():
    """One shard of BASELINE.json config 5 at its stated size: N = 262,144 members over 8 GPUs, so this GPU holds
    observer rows [0, 32,768) (the canonical split) with every dense cell, the message pool and the snapshot slots
    of DESIGN.md §2. The reference keeps the disseminator and timers as maps (disseminator.go:47,
    state_transitions.go:52); here they are dense cells, and this checks on hardware that the budget fits with at
    least 10 % headroom, and that a 262,144-member row's checksum (a 10 MB string) equals Fingerprint32 of the
    reference's string rebuilt from the row (memberlist.go:106-128)."""
    import ctypes

    from oracle_ffi import fingerprint32

    # (the device's memory through the HIP runtime the engine uses: torch's own runtime may refuse the GPU once the
    # engine's has initialised it in this process)
    hip = ctypes.CDLL("libamdhip64.so")
    free_b, total_b = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)) == 0
    total = total_b.value
    if total < 280e9:
        pytest.skip(f"needs a 288 GB MI355X ({total / 1e9:.0f} GB visible)")
    n, shard = 262144, (0, 32768)
    eng = swimsim.Cluster(n, observer_range=shard)
    try:
        m = eng.memory()
        np_ = n
        rows = shard[1] - shard[0]
        assert m["row_words"] == rows * np_ * 4
        assert m["dissemination"] >= rows * np_ * 8 and m["timers"] >= rows * np_ * 9
        assert m["total"] <= 0.90 * total, f"{m['total'] / 1e9:.1f} GB of {total / 1e9:.1f} GB: < 10 % headroom"
        assert m["message_pool"] >= 2 * rows * 26214 * 16 // 2   # one burst's requests + responses
        cs = eng.checksums()
        for o in (0, rows - 1):
            st, inc = eng.row(o)
            assert (st == swimsim.ALIVE).all()
            s = "".join(f"{swimsim.address_of(k)}alive{swimsim.T0_MS};" for k in range(n))
            assert int(cs[o]) == fingerprint32(s.encode()), f"observer {o}"
        print(f"config5 shard {shard} of N={n}: {m}")
    finally:
        eng.close()


def test_message_pool_must_hold_the_longest_message_per_sub_pool():
    """pool_alloc's 64 sub-pools each take a whole message; a message has up to N records (no per-message cap,
    SURVEY.md §0.2), so a caller-set pool below 64 x N records is refused at create time"""
    n = 1024
    with pytest.raises(swimsim.SwimsimError):
        swimsim.Cluster(n, message_pool_bytes=64 * n * 16 - 16)
    eng = swimsim.Cluster(n, message_pool_bytes=64 * n * 16)
    eng.step(3)
    eng.close()
