"""Per-kernel, per-launch PMC figures from rocprofv3 --pmc passes of bench.py (one directory per pass).

usage: python tools/pmc_summary.py [--workload MEMBERS:STEPS:WARMUP:GPUS[:NAME]] [--window] <out.json> <pass_dir> [<pass_dir> ...]
--workload records the bench.py command the passes profiled (bench.py uses the summary only for that workload).
--window keeps only the dispatches between the first and the last k_profile_mark dispatch of each pass (bench.py
marks its timed rounds), so the per-launch figures cover exactly the launches its HIP-event timings cover.
Every counter of every pass is averaged per launch of each kernel. FETCH_SIZE and WRITE_SIZE are in
KiB (TCC_EA0_RDREQ/WRREQ-derived) and are reported as bytes. MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced 16-B/lane streaming read (doubled here as
fetch_bytes_wide_corrected); other access widths are uncalibrated, so the raw figure is kept beside it.
SQ_INSTS_* count wave-instructions; GRBM_GUI_ACTIVE is summed over the 8 XCDs (÷ 8 = GPU cycles).
"""
import collections
import csv
import json
import sys


def load(path, agg, window):
    rows = list(csv.DictReader(open(f"{path}/run_counter_collection.csv")))
    lo, hi = -1, float("inf")
    if window:
        marks = sorted(int(x["Dispatch_Id"]) for x in rows if "k_profile_mark" in x["Kernel_Name"])
        if len(marks) < 2:
            raise SystemExit(f"{path}: --window needs two k_profile_mark dispatches, found {len(marks)}")
        lo, hi = marks[0], marks[-1]
    for x in rows:
        if not lo < int(x["Dispatch_Id"]) < hi:
            continue
        k = x["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        c = x["Counter_Name"]
        agg[k][c][0].add(x["Dispatch_Id"])
        agg[k][c][1] += float(x["Counter_Value"])


def main():
    argv = sys.argv[1:]
    workload = None
    if argv and argv[0] == "--workload":
        f = argv[1].split(":")
        m, st, w, g = (int(x) for x in f[:4])
        workload = {"members": m, "steps": st, "warmup": w, "gpus": g}
        if len(f) > 4 and f[4] != "config3":                      # (bench.py --workload; config3 is the default)
            workload["workload"] = f[4]
        argv = argv[2:]
    window = False
    if argv and argv[0] == "--window":
        window = True
        argv = argv[1:]
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: [set(), 0.0]))
    for p in argv[1:]:
        load(p, agg, window)
    out = {"_workload": workload, "_window": "between k_profile_mark dispatches (bench.py timed rounds)" if window else None}
    for k in sorted(agg):
        e = {}
        for c, (ids, v) in agg[k].items():
            n = max(len(ids), 1)
            e["launches"] = max(e.get("launches", 0), n)
            if c == "FETCH_SIZE":
                e["fetch_bytes_per_launch"] = v * 1024.0 / n
                e["fetch_bytes_wide_corrected_per_launch"] = 2 * v * 1024.0 / n
            elif c == "WRITE_SIZE":
                e["write_bytes_per_launch"] = v * 1024.0 / n
            else:
                e[c.lower() + "_per_launch"] = v / n
        out[k] = e
    json.dump(out, open(argv[0], "w"), indent=1)


if __name__ == "__main__":
    main()
