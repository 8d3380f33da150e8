import sys, json
sys.path.insert(0, "ringpop-go_amd")
import swimsim
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
c = swimsim.Cluster(n, observer_range=(0, min(n, 16384)))
out = {}
for rows in (64, 1024, 4096, 16384):
    if rows > c.nl:
        continue
    for mode in (0, 1, 2):
        out[f"rows{rows}_mode{mode}"] = round(c.bench_checksum(rows, mode, reps=2), 3)
print(json.dumps(out))
