"""BASELINE.json config 5 (large incarnation bursts) beyond its reduced-size parity case: the dense-snapshot
budget. A reincarnation burst dirties many rows at once, and lazy C_o (k_issue) would take one dense snapshot
per dirty sender. When the snapshot slots could not hold them, the engine hashes the dirty senders before issue
instead (bound_lazy_snapshots): exact either way. These tests force a small slot pool so that the
fallback runs, and compare every round with the oracle."""
import os

import pytest

import swimsim
from swimsim import workloads as W
from test_engine_parity import make_pair, run_parity

pytestmark = pytest.mark.gpu


def _small_pool_pair(n, cap=64):
    os.environ["SWIMSIM_DENSE_CAP"] = str(cap)
    try:
        return make_pair(n)
    finally:
        del os.environ["SWIMSIM_DENSE_CAP"]


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
