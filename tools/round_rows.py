"""Per-round checksum work of config 3 (diagnostic, not the bench): the cluster steps one round per call and prints,
for every round, the rows each checksum family hashed and its kernel time (kernel_times / kernel_units deltas).
One round per call makes every side-stream launch finish inside its own round; the row counts are the bench's.
Usage: round_rows.py [N] [rounds]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 25
wl = W.config3(n=n, rounds=rounds, kill_round=10)
c = swimsim.Cluster(n)
c.enable_timing(True)
prev_t, prev_u = {}, {}
for r in range(rounds):
    c.step(1, wl.events_for(r))
    kt, ku = c.kernel_times(), c.kernel_units()
    row = {"round": r}
    for fam in ("checksum_wide", "checksum_narrow", "checksum_delta_scan", "checksum_prep"):
        if fam not in kt:
            continue
        ms = kt[fam]["avg_ms"] * kt[fam]["launches"]
        p = prev_t.get(fam, (0.0, 0))
        dl = kt[fam]["launches"] - p[1]
        if dl:
            row[fam] = {"launches": dl, "ms": round(ms - p[0], 3)}
        prev_t[fam] = (ms, kt[fam]["launches"])
    for u in ("cs_rows_wide", "cs_rows_narrow", "cs_dup_rows"):
        row[u] = int(ku.get(u, 0) - prev_u.get(u, 0))
        prev_u[u] = ku.get(u, 0)
    print(json.dumps(row), flush=True)
