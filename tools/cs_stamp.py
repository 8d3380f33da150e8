"""Per-role busy cycles of the wide checksum kernel (diagnostic; diagnostics library, modes 62/63 = k_checksum6 with
s_memtime stamps, one or two hasher waves): config 3 at N members run to round R (real cascade rows), then each
mode is launched over the first `rows` rows; every wave sums its busy shader cycles per step (from the barrier's
release to its arrival at the next one) and the result is printed per workgroup-step, beside the launch time.
Usage: SWIMSIM_LIBRARY=tools/libswimsim_diag.so cs_stamp.py N R modes rows,rows,..."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n, R = int(sys.argv[1]), int(sys.argv[2])
modes = [int(x) for x in sys.argv[3].split(",")]
rows_list = [int(x) for x in sys.argv[4].split(",")]
wl = W.config3(n=n, rounds=R + 1, kill_round=10)
c = swimsim.Cluster(n)
for r in range(R):
    c.step(1, wl.events_for(r))
steps = (n + 15) // 16 * 4
out = {"n": n, "round": R, "steps_per_row": steps}
for rows in rows_list:
    for mode in modes:
        u0 = c.kernel_units()
        ms = c.bench_checksum(rows, mode, reps=1)               # warm-up + 1 timed launch: 2 launches stamped
        u1 = c.kernel_units()
        wg_steps = 2 * ((rows + 63) // 64) * steps
        per = {k: round((u1[k] - u0[k]) / wg_steps, 1) for k in ("diag_stamp0", "diag_stamp1", "diag_stamp2")}
        per["formatter_loop_cycles_per_step"] = round((u1["diag_stamp3"] - u0["diag_stamp3"]) / wg_steps, 1)
        out[f"rows{rows}_mode{mode}"] = {"ms": round(ms, 3), "busy_cycles_per_step": per,
                                         "launch_cycles_per_step_at_2.4GHz": round(ms * 1e-3 * 2.4e9 / steps, 1)}
        print(json.dumps(out), flush=True)
