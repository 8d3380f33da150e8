"""Generates the per-round oracle fixtures of BASELINE.json's configs at their full sizes:

  config2_n4096.json   4,096 members, 1 % kill/revive churn per round, 200 rounds (configs[1])
  config4_n16384.json  16,384 members, halves partitioned for rounds 0-59, Heal on observer 0 at rounds 60 and
                       80, run until the reference's convergence criterion holds (test_utils.go:164-199: no live
                       node has changes and all live checksums are equal) (configs[3])
  config5_n4096.json   4,096 members, 10 % of them Reincarnate every 20 rounds, 100 rounds (configs[4] at the
                       largest size the oracle runs in minutes)
  selfstart_n16384.json 16,384 members starting self-only, members 0 and 1 seeded at every node by MakeChange, 40
                       rounds: the full-sync and reverse-full-sync paths at size (counters full_syncs, rfs_done > 0)
  config3_n65536.json  bench.py's own workload: 65,536 members, 655 killed at round 10 (Philox seed 11), rounds
                       0-99: steady state, the kill, the suspect wave and the whole faulty wave (r >= 35)
                       (configs[2]; dense oracle rows ~39 GB, generated in the 62-GB build container)

Each per-round record holds: the round, sha256 of the checksum vector (uint32 little-endian, observer order),
sha256 of the phase-S ping targets (int32 little-endian), the three canonical state digests (member rows,
dissemination buffers, timer tables; or_digest), the protocol counters and whether the cluster has converged.

The oracle is oracle/swim_oracle.c built with OpenMP over observers (oracle/build/libswim_oracle_omp.so);
tests/test_oracle_kats.py::test_openmp_oracle_equals_single_thread pins that build to the single-threaded one.
TEST INFRASTRUCTURE ONLY: tests/test_parity_at_size.py compares the MI355X engine with these files on the GPU.

usage: python tests/golden/make_size_fixtures.py {config2|config4|config5|config3|selfstart} [threads]"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("OMP_NUM_THREADS", sys.argv[2] if len(sys.argv) > 2 else "8")
os.environ["ORACLE_LIB"] = os.path.join(REPO, "oracle", "build", "libswim_oracle_omp.so")
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "ringpop-go_amd"))

import numpy as np  # noqa: E402

from oracle_ffi import OracleSim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

CONFIGS = {
    # name: (workload, stop at convergence (after the last scheduled event), output file)
    "config2": (lambda: W.config2(n=4096, rounds=200), False, "config2_n4096.json"),
    "config4": (lambda: W.config4(n=16384, rounds=260), True, "config4_n16384.json"),
    "config5": (lambda: W.config5(n=4096, rounds=100), False, "config5_n4096.json"),
    "config3": (lambda: W.config3(n=65536, rounds=100, kill_round=10), False, "config3_n65536.json"),
    "selfstart": (lambda: W.selfstart(n=16384, seeds=2, rounds=40), False, "selfstart_n16384.json"),
}


def seed_rows(sim, wl, alive=0):
    """the workload's MakeChange seeding before round 0 (oracle or engine: both take make_change(o, m, inc, status))"""
    t0 = 1_500_000_000_000
    for o in range(wl.n):
        for m in wl.seed_members:
            if m != o:
                sim.make_change(o, m, t0, alive)


def sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a).astype(dt).tobytes()).hexdigest()


def record(ora, r, conv):
    return {"round": r, "checksums_sha256": sha(ora.checksums(), "<u4"),
            "targets_sha256": sha(ora.last_targets(), "<i4"),
            "digest": [f"{x:016x}" for x in ora.digest()], "counters": ora.counters(), "converged": conv}


def generate(name):
    make, until_conv, fname = CONFIGS[name]
    wl = make()
    last_event = max((e[0] for e in wl.events), default=-1)
    ora = OracleSim(wl.n, init=wl.init)
    seed_rows(ora, wl)
    recs, t0 = [], time.time()
    for r in range(wl.rounds):
        ora.step(wl.events_for(r))
        conv = until_conv and r > last_event and ora.converged()
        recs.append(record(ora, r, conv))
        print(f"{name} r={r} {time.time() - t0:.0f}s conv={conv}", file=sys.stderr, flush=True)
        if conv:
            break
    out = {"workload": wl.name, "n": wl.n, "events": wl.description, "rounds": len(recs), "records": recs,
           "generator": "tests/golden/make_size_fixtures.py %s (oracle/swim_oracle.c, OpenMP build)" % name}
    with open(os.path.join(HERE, fname), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    generate(sys.argv[1])
