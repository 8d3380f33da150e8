"""Checksum-kernel microbench (diagnostic, not the bench): average ms per launch of k_checksum over the
first `rows` observer rows of a converged N-member cluster, mode 0 = full kernel, 1 = hash waves only,
2 = formatter wave only, 4 = barrier skeleton, 5 = formatter loads and positions only (modes 1, 2, 4
and 5 leave garbage checksums), 6 = the 16-row narrow kernel. With a 5th argument "verify", rows are
perturbed first (one suspect each) and the checksums of mode 6 are compared with mode 0's."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rows_list = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 1024, 4096, 16384]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
modes = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1, 2]
verify = len(sys.argv) > 5 and sys.argv[5] == "verify"
c = swimsim.Cluster(n, observer_range=(0, min(n, max(rows_list))))
if verify:
    for o in range(min(n, max(rows_list), 4096)):
        c.make_change(o, (o * 7919 + 1) % n, swimsim.T0_MS + 200 * (1 + o % 7), 1)
    c.checksums()
out = {}
for rows in rows_list:
    ref = None
    for mode in modes:
        out[f"rows{rows}_mode{mode}"] = round(c.bench_checksum(rows, mode, reps=reps), 3)
        if verify and mode in (0, 6, 20, 21, 30, 33, 44, 45):
            cs = c.checksums()[:rows].copy()
            if ref is None:
                ref = cs
            else:
                out[f"rows{rows}_mode{mode}_mismatch"] = int((cs != ref).sum())
print(json.dumps(out))
