"""Hot columns: per-row compact copies of the row words and dissemination cells of the members that sit
in dissemination buffers, read by issue, merge and bump instead of one scattered sector per member. They are copies,
so no result may depend on them (the slot is a hot member's dissemination cell, written back to the dense
array before the slots are dropped or a row is read back): these tests run workloads with the columns off (swimsim_tuning.hot_slots = 0), with a few
slots that overflow (members beyond them stay on the dense path) and with the default, and require every round to
match the oracle or the column-free engine bit for bit."""

import pytest

import swimsim
from swimsim import workloads as W
from test_engine_parity import make_pair, run_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("slots", [0, 64])
def test_churn_parity_with_few_or_no_hot_slots(slots):
    # config 2's churn brings new members into buffers every round: 64 slots fill up and later members stay dense
    wl = W.config2(n=256, rounds=40)
    eng, ora = make_pair(wl.n, tuning={"hot_slots": slots})
    run_parity(eng, ora, wl.n, wl.rounds, wl.events)


def test_cascade_same_with_and_without_hot_columns():
    wl = W.config3(n=4096, rounds=45, kill_round=3)
    on = swimsim.Cluster(wl.n)
    off = swimsim.Cluster(wl.n, tuning={"hot_slots": 0})
    try:
        for r in range(wl.rounds):
            ev = wl.events_for(r)
            on.step(1, ev)
            off.step(1, ev)
            assert (on.checksums() == off.checksums()).all(), f"round {r}: checksums differ"
            assert on.digest() == off.digest(), f"round {r}: state digests differ"
            assert on.counters() == off.counters(), f"round {r}: counters differ"
            if r % 5 == 4:                                   # host read-back of the cells (hot slots flushed first)
                for o in (0, 1, 777, wl.n - 1):
                    assert on.changes(o) == off.changes(o), f"round {r}: row {o} dissemination cells"
        assert on.counters()["timers_fired"] > 0
    finally:
        on.close()
        off.close()


def test_join_and_raw_writes_reset_the_columns():
    # swimsim_set_row / set_member write rows directly; the columns are dropped and rebuilt from later entries
    wl = W.config3(n=512, rounds=30, kill_round=2)
    eng, ora = make_pair(wl.n)
    run_parity(eng, ora, wl.n, 12, wl.events)
    st, inc = ora.row(7)
    eng.set_row(7, st, inc)
    run_parity(eng, ora, wl.n, wl.rounds - 12, wl.events)
