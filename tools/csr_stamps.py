"""Diagnostics: where k_csr's loop spends its cycles (build with -DCSR_DIAG_STAMP, loaded through SWIMSIM_LIBRARY):
config 3 at N members to round R, then swimsim_bench_checksum mode 5 (the reference-row path) over `rows` rows; prints
the summed per-wave shader-clock cycles of the chain, the staging + preparation, the barrier and the whole loop.
Usage: csr_stamps.py N R rows"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n, R, rows = (int(x) for x in sys.argv[1:4])
wl = W.config3(n=n, rounds=R + 1, kill_round=10)
c = swimsim.Cluster(n)
for r in range(R):
    c.step(1, wl.events_for(r))
c.bench_checksum(rows, 5, reps=1)
c.enable_timing(True)
ms = c.bench_checksum(rows, 5, reps=1)
ku = c.kernel_units()
st = [ku.get(f"diag_stamp{i}", 0) for i in range(4)]
tot = st[3] or 1
print(json.dumps({"rows": rows, "ms": ms, "cycles": st, "share": {k: round(st[i] / tot, 3) for i, k in
                                                                  enumerate(["chain", "prep", "barrier", "loop"])}}))
