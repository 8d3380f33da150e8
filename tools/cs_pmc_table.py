"""Diagnostics: per-dispatch SQ counters of the checksum kernels from tools/gpu_cs_pmc.sh (dispatch order =
tools/cs_bench.py's launch order: warm-up + reps per (rows, mode))."""
import collections
import csv
import sys

rows = collections.defaultdict(dict)
names = {}
for d in sys.argv[1:]:
    for x in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = x["Kernel_Name"]
        if "checksum" not in k:
            continue
        i = int(x["Dispatch_Id"])
        names[i] = (k.split("(")[0].replace("void swimdev::", ""), x.get("Grid_Size", ""))
        rows[(d, i)][x["Counter_Name"]] = float(x["Counter_Value"])
by = collections.defaultdict(dict)
for (d, i), v in rows.items():
    by[i].update(v)
for i in sorted(by):
    v = by[i]
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    print(i, names[i], {k: (f"{val / wc:.3f}" if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else f"{val:.3e}") for k, val in sorted(v.items())})
