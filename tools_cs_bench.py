"""Checksum-kernel microbench (diagnostic, not the bench): average ms per launch of k_checksum over the
first `rows` observer rows of a converged N-member cluster, mode 0 = full kernel, 1 = hash waves only,
2 = formatter wave only, 4 = barrier skeleton, 5 = formatter loads and positions only (modes 1, 2, 4
and 5 leave garbage checksums)."""
import json
import sys

sys.path.insert(0, "ringpop-go_amd")
import swimsim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rows_list = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 1024, 4096, 16384]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
modes = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1, 2]
c = swimsim.Cluster(n, observer_range=(0, min(n, max(rows_list))))
out = {}
for rows in rows_list:
    for mode in modes:
        out[f"rows{rows}_mode{mode}"] = round(c.bench_checksum(rows, mode, reps=reps), 3)
print(json.dumps(out))
