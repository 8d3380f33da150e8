"""Per-round timeline of a rocprofv3 --kernel-trace run of bench.py, cut to the timed window (the dispatches between
the first and the last k_profile_mark): a round starts at its k_timers dispatch. For every round: wall time, the time
some kernel was running (union of the dispatch intervals), the idle gaps (host work between launches), and the time
of the main families (by the round their dispatch started in), where the side-stream checksum launches are reported
apart with the part of them that overlapped another kernel (of any round).

usage: python tools/prof_timeline.py <run_kernel_trace.csv> [out.txt]"""
import collections
import csv
import sys

FAMILIES = [("k_csr3", "cs_csr3"), ("k_csd_scan", "cs_scan"), ("k_csr_rec", "cs_rec"), ("k_checksum3", "cs_wide"), ("k_checksum_q16", "cs_narrow"), ("k_recv", "recv"), ("k_resp", "resp"),
            ("k_issue", "issue"), ("k_fp_", "fp"), ("rocprim", "sort"), ("hipcub", "sort")]


COLS = ("cs_csr3", "cs_scan", "cs_rec", "cs_wide", "cs_narrow", "overlap", "recv", "resp", "issue", "fp", "sort",
        "other")


def family(name):
    for key, fam in FAMILIES:
        if key in name:
            return fam
    return "other"


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marks = sorted(int(r["Dispatch_Id"]) for r in rows if "k_profile_mark" in r["Kernel_Name"])
    lo, hi = marks[0], marks[-1]
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Dispatch_Id"]))
                 for r in rows if lo < int(r["Dispatch_Id"]) < hi), key=lambda k: k[0])
    mark_t = sorted(int(r["Start_Timestamp"]) for r in rows if "k_profile_mark" in r["Kernel_Name"])
    starts = [k[0] for k in ks if "k_timers" in k[2]] + [mark_t[-1]]
    out = []
    hdr = f"{'round':>5} {'wall_ms':>8} {'busy_ms':>8} {'idle_ms':>8} " + " ".join(
        f"{f:>9}" for f in COLS)
    out.append(hdr)
    tot = collections.Counter()
    for i in range(len(starts) - 1):
        a, b = starts[i], starts[i + 1]
        sel = [k for k in ks if a <= k[0] < b]
        busy = union([(max(s, a), min(e, b)) for s, e, _, _ in ks if s < b and e > a])
        fam = collections.Counter()
        for s, e, n, _ in sel:
            fam[family(n)] += e - s
        narrow = [(s, e) for s, e, n, _ in sel if family(n) == "cs_narrow"]
        others = [(s, e) for s, e, n, _ in ks if family(n) != "cs_narrow"]
        ov = 0
        for s, e in narrow:
            ov += union([(max(s, x), min(e, y)) for x, y in others if x < e and y > s])
        wall = b - a
        row = {"wall": wall, "busy": busy, "idle": wall - busy, "overlap": ov, **fam}
        tot.update(row)
        out.append(f"{i:>5} {wall / 1e6:8.3f} {busy / 1e6:8.3f} {(wall - busy) / 1e6:8.3f} " + " ".join(
            f"{row.get(f, 0) / 1e6:9.3f}" for f in COLS))
    out.append(f"{'sum':>5} {tot['wall'] / 1e6:8.3f} {tot['busy'] / 1e6:8.3f} {tot['idle'] / 1e6:8.3f} " + " ".join(
        f"{tot.get(f, 0) / 1e6:9.3f}" for f in COLS))
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main()
