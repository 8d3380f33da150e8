"""Which kernels a launch waited behind: for every dispatch of a kernel family (default k_csr3) in a rocprofv3 kernel
trace of bench.py, its start and end relative to the window, and every dispatch of the other families (default the
side-stream checksum kernels) whose interval overlaps it or ends within 0.5 ms before it starts.

usage: python tools/trace_overlap.py <run_kernel_trace.csv[.gz]> [target] [others, comma separated]"""
import csv
import gzip
import sys


def main():
    path = sys.argv[1]
    target = sys.argv[2] if len(sys.argv) > 2 else "k_csr3"
    others = (sys.argv[3] if len(sys.argv) > 3 else "k_checksum_q16,k_csr3,k_csd_scan,k_csr_rec").split(",")
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = list(csv.DictReader(f))
    t0 = min(int(r["Start_Timestamp"]) for r in rows if "k_profile_mark" in r["Kernel_Name"])
    ks = sorted((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"].split("(")[0],
                 int(r["Dispatch_Id"])) for r in rows)
    for s, e, n, i in ks:
        if target not in n or s < 0:
            continue
        print(f"{n[:40]:40s} #{i:6d} {s / 1e6:9.3f} .. {e / 1e6:9.3f} ms ({(e - s) / 1e6:.3f})")
        for s2, e2, n2, i2 in ks:
            if i2 == i or not any(o in n2 for o in others):
                continue
            if s2 < e and e2 > s - 500_000:
                print(f"    {n2[:36]:36s} #{i2:6d} {s2 / 1e6:9.3f} .. {e2 / 1e6:9.3f} ({(e2 - s2) / 1e6:.3f})")


if __name__ == "__main__":
    main()
