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
st = [ku.get(f"diag_stamp{i}", 0) for i in range(8)]
tot = st[3] or 1
# k_csr3: 0-3 the g/f chain waves (chain, waiting for the stagers, codes, whole loop), 4-7 the stagers (waiting for the
# chains, the record loads (vmcnt), rows' codes and exceptions, hand-over), each as a share of the chain waves' loop
names = ["chain", "wait", "codes", "loop", "s_wait", "s_recload", "s_prep", "s_signal"]
print(json.dumps({"round": R, "rows": rows, "ms": ms, "cycles": st, "share": {k: round(st[i] / tot, 3) for i, k in
                                                                              enumerate(names)}}))
