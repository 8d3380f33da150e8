"""The reference-row checksum path (tools/diag/swimsim_checksum_delta.hip: k_csd_scan + k_cs_delta) against the CPU
oracle. The path lives in the diagnostics library only (round 4: it did not pay over the cascade), so
these tests run when that library is the one loaded:
    SWIMSIM_LIBRARY=tools/libswimsim_diag.so python -m pytest tools/diag/test_cs_delta.py
and skip otherwise. (Kept here, beside the diagnostics sources, since round 6: in tests/ they always skipped on the
product library.)

The path is forced onto every phase-C launch of at least 1,024 rows (SWIMSIM_CS_DELTA=2, synchronous phase C so
every launch goes through it) at sizes where the oracle runs every round: the cascade (rows a few records apart),
churn (incarnation bumps: longer and shorter records), a partition (rows half a membership apart: the workgroup
plans fail and the rows go to the production kernels) and a self-only start. Bit-exact per round, as every
other checksum kernel (memberlist.go:83-128). """
import os
import sys

import numpy as np
import pytest

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(_REPO, "tests"), os.path.join(_REPO, "ringpop-go_amd")]

from oracle_ffi import OracleSim  # noqa: E402
import swimsim
from swimsim import workloads as W

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif("libswimsim_diag" not in os.environ.get("SWIMSIM_LIBRARY", ""),
                                 reason="reference-row path: diagnostics library only (SWIMSIM_LIBRARY=tools/libswimsim_diag.so)")]


def forced(n, **kw):
    old = {k: os.environ.get(k) for k in ("SWIMSIM_CS_DELTA", "SWIMSIM_CS_DELTA_MAXDIFF")}
    try:
        os.environ["SWIMSIM_CS_DELTA"] = "2"
        os.environ["SWIMSIM_CS_DELTA_MAXDIFF"] = str(kw.pop("maxdiff", 0))
        return swimsim.Cluster(n, tuning={"cs_async": 0}, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_vs_oracle(wl, rounds, init="converged"):
    eng = forced(wl.n, init=init)
    ora = OracleSim(wl.n, init=init)
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
    assert st["fallback_rows"] <= st["delta_launches"] * 64, st


def test_churn_n2048_every_round():
    wl = W.config2(n=2048, rounds=40)
    eng = run_vs_oracle(wl, 40)
    st = eng.checksum_path_stats()
    print("churn n2048", st)
    assert st["delta_launches"] >= 5, st


def test_partition_n2048_falls_back_exactly():
    wl = W.config4(n=2048, rounds=90)
    eng = run_vs_oracle(wl, 90)
    st = eng.checksum_path_stats()
    print("partition n2048", st)
    assert st["delta_launches"] >= 1, st


def test_bench_checksum_mode3_on_real_cascade_rows():
    n = 4096
    wl = W.config3(n=n, rounds=30, kill_round=10)
    c = swimsim.Cluster(n)
    for r in range(18):
        c.step(1, wl.events_for(r))
    ref = c.checksums().copy()
    for rows in (1024, 2048, n):
        c.bench_checksum(rows, 3, reps=1)
        got = c.checksums()
        assert (got[:rows] == ref[:rows]).all(), f"{rows} rows: {(got[:rows] != ref[:rows]).sum()} differ"
    print("real rows n4096", c.checksum_path_stats())


def test_incarnation_bursts_n2048_every_round():
    wl = W.config5(n=2048, rounds=45, every=20)
    eng = run_vs_oracle(wl, 45)
    st = eng.checksum_path_stats()
    print("bursts n2048", st)
    assert st["delta_launches"] >= 3, st


def test_predictor_declines_far_rows_and_stays_exact():
    """with the default threshold the path declines the partition's launches (rows half a membership apart) and the
    production kernels hash them; the cascade's early launches (rows a few members apart) take the path"""
    wl = W.config4(n=2048, rounds=70)
    eng = forced(wl.n, maxdiff=12)
    ora = OracleSim(wl.n)
    for r in range(70):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
        assert (eng.checksums() == ora.checksums()).all(), f"round {r}"
    st = eng.checksum_path_stats()
    print("partition predictor", st)
    assert st["reasons"]["declined_launches"] >= 1, st
