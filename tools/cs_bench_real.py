"""Checksum-kernel microbench on real cascade rows (diagnostic, not the bench): config 3 at N members is run to
round R (inside the suspect wave, where every row is dirty and the rows differ in which suspects they hold),
then the wide checksum launch is timed over all rows for each mode (swimsim_bench_checksum modes: 21 =
k_checksum3). Usage: cs_bench_real.py N R modes reps"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
R = int(sys.argv[2]) if len(sys.argv) > 2 else 18
modes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [21]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
wl = W.config3(n=n, rounds=R + 1, kill_round=10)
c = swimsim.Cluster(n)
for r in range(R):
    c.step(1, wl.events_for(r))
ref = c.checksums().copy()
out = {"n": n, "round": R}
for mode in modes:
    out[f"mode{mode}"] = round(c.bench_checksum(n, mode, reps=reps), 3)
    out[f"mode{mode}_mismatch"] = int((c.checksums() != ref).sum())
print(json.dumps(out))
