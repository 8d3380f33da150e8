"""Summarise tools/gpu_r6_curve.sh output (gpurun_out/cs/curve_r*.json, curve_big_r*.json) into one JSON: per cascade
round, per row count, the launch time of each checksum mode (0 production choice, 5 reference-row path on the main
stream, 6 the same on the side stream with its own buffer set) and the mismatch count against the engine's checksums.
usage: python tools/curve_summary.py <out.json>"""
import glob
import json
import re
import sys

out = {"what": "checksum launch time on real cascade rows of config 3 at 65,536 members (tools/cs_bench_real.py), the first "
               "R rows of the round; modes: 0 production choice, 5 reference-row path on the main stream, 6 the same on "
               "the side stream (csr2 buffer set, at most 12,288 rows)", "rounds": {}}
for f in sorted(glob.glob("gpurun_out/cs/curve_*r*.json")):
    R = int(re.search(r"_r(\d+)\.json", f).group(1))
    lines = [l for l in open(f).read().splitlines() if l.strip()]
    if not lines:
        continue
    d = json.loads(lines[-1])
    row = out["rounds"].setdefault(str(R), {})
    for k, v in d.items():
        m = re.match(r"rows(\d+)_mode(\d+)_(ms|mismatch)$", k)
        if m:
            row.setdefault(m.group(1), {})[f"mode{m.group(2)}_{m.group(3)}"] = v
json.dump(out, open(sys.argv[1], "w"), indent=1)
for R, rows in sorted(out["rounds"].items(), key=lambda kv: int(kv[0])):
    print(R, {n: {k: v for k, v in e.items() if k.endswith("_ms")} for n, e in sorted(rows.items(), key=lambda kv: int(kv[0]))},
          "mismatches", sum(v for e in rows.values() for k, v in e.items() if k.endswith("mismatch")))
