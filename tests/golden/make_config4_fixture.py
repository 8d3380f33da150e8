"""Generates tests/golden/config4_n16384.json: per-round oracle records of BASELINE.json config 4 at its full
size (16,384 members, halves partitioned for rounds 0-59, Heal on observer 0 at rounds 60 and 80), run until the
reference's convergence criterion holds (test_utils.go:164-199: no live node has changes and all live checksums
are equal). Each record: round, sha256 of the checksum vector (uint32 little-endian, observer order), the three
canonical state digests, the protocol counters and whether the cluster converged.

The oracle is oracle/swim_oracle.c built with OpenMP over observers (oracle/build/libswim_oracle_omp.so);
tests/test_oracle_kats.py::test_openmp_oracle_equals_single_thread pins that build to the single-threaded one.
TEST INFRASTRUCTURE: tests/test_parity_at_size.py compares the engine with this file on the GPU.

usage: python tests/golden/make_config4_fixture.py [threads]"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("OMP_NUM_THREADS", sys.argv[1] if len(sys.argv) > 1 else "8")
os.environ["ORACLE_LIB"] = os.path.join(REPO, "oracle", "build", "libswim_oracle_omp.so")
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "ringpop-go_amd"))

from oracle_ffi import OracleSim, lib  # noqa: E402
from swimsim import workloads as W  # noqa: E402

N, MAX_ROUNDS = 16384, 260


def cs_hash(ora, n):
    import numpy as np
    cs = np.zeros(n, np.uint32)
    for o in range(n):
        cs[o] = lib().or_checksum(ora.h, o)
    return hashlib.sha256(cs.astype("<u4").tobytes()).hexdigest()


def main():
    wl = W.config4(n=N, rounds=MAX_ROUNDS)
    ora = OracleSim(N)
    recs, t0 = [], time.time()
    for r in range(MAX_ROUNDS):
        ora.step(wl.events_for(r))
        d = ora.digest()
        conv = r >= 80 and ora.converged()
        recs.append({"round": r, "checksums_sha256": cs_hash(ora, N), "digest": [f"{x:016x}" for x in d],
                     "counters": ora.counters(), "converged": conv})
        print(f"r={r} {time.time() - t0:.0f}s conv={conv}", file=sys.stderr, flush=True)
        if conv:
            break
    out = {"workload": wl.name, "n": N, "events": wl.description, "rounds": len(recs), "records": recs,
           "generator": "tests/golden/make_config4_fixture.py (oracle/swim_oracle.c, OpenMP build)"}
    with open(os.path.join(HERE, "config4_n16384.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
