"""Per-kernel launch statistics of a rocprofv3 --kernel-trace run, cut to the dispatches between the first and the
last k_profile_mark (bench.py marks its timed rounds), in the format of rocprofv3's kernel_stats.csv
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs). The whole-run --stats summary includes the
warm-up rounds and the initial hash of every row; this one covers exactly the launches the bench line's HIP-event
averages cover.

usage: python tools/prof_window.py <run_kernel_trace.csv> <out.csv>"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marks = sorted(int(r["Dispatch_Id"]) for r in rows if "k_profile_mark" in r["Kernel_Name"])
    if len(marks) < 2:
        raise SystemExit(f"need two k_profile_mark dispatches, found {len(marks)}")
    lo, hi = marks[0], marks[-1]
    d = collections.defaultdict(list)
    for r in rows:
        if lo < int(r["Dispatch_Id"]) < hi:
            d[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in d.values())
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])


if __name__ == "__main__":
    main()
