"""Checksum-kernel microbench on real cascade rows (diagnostic, not the bench): config 3 at N members is run to
round R (inside the suspect wave, where every row is dirty and the rows differ in which suspects they hold),
then each checksum mode is timed over the first `rows` rows for every row count given (swimsim_bench_checksum
modes: 0 = the production choice for that many rows, 1 = k_checksum3, 2 = k_checksum_q16; the diagnostics library
(SWIMSIM_LIBRARY=tools/libswimsim_diag.so) adds 21 = k_checksum3, 50/51 = k_checksum5 with the record-tail prefetch
1/2 steps ahead, ...). Every launch's checksums are compared with the engine's own (mismatch counts).
Usage: cs_bench_real.py N R modes reps [rows,rows,...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
R = int(sys.argv[2]) if len(sys.argv) > 2 else 18
modes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
rows_list = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [n]
wl = W.config3(n=n, rounds=R + 1, kill_round=10)
# CS_TUNING='{"fault_inject": 512}' (a JSON object of swimsim_tuning fields): an engine variant, same results
c = swimsim.Cluster(n, tuning=json.loads(os.environ["CS_TUNING"]) if os.environ.get("CS_TUNING") else None)
for r in range(R):
    c.step(1, wl.events_for(r))
ref = c.checksums().copy()
out = {"n": n, "round": R, "library": os.path.basename(os.environ.get("SWIMSIM_LIBRARY", "libswimsim.so")),
       "tuning": os.environ.get("CS_TUNING", "")}
for rows in rows_list:
    for mode in modes:
        out[f"rows{rows}_mode{mode}_ms"] = round(c.bench_checksum(rows, mode, reps=reps), 3)
        out[f"rows{rows}_mode{mode}_mismatch"] = int((c.checksums()[:rows] != ref[:rows]).sum())
        if mode in (3, 5):
            out[f"rows{rows}_mode{mode}_path"] = c.checksum_path_stats()
        if mode == 3:
            ku = c.kernel_units()
            out["diag"] = [hex(int(ku.get(f"diag_stamp{i}", 0))) for i in range(4)]
        print(json.dumps(out), flush=True)
