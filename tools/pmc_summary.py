"""Per-kernel, per-launch HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>
FETCH_SIZE and WRITE_SIZE are in KiB (TCC_EA0_RDREQ/WRREQ-derived). MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced 16-B/lane streaming read (doubled here as
fetch_bytes_wide_corrected); other access widths are uncalibrated, so the raw figure is kept beside it.
"""
import collections
import csv
import json
import sys


def load(path):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for x in csv.DictReader(open(f"{path}/run_counter_collection.csv")):
        k = x["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        agg[k][0] += 1
        agg[k][1] += float(x["Counter_Value"]) * 1024.0
    return agg


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    out = {}
    for k in sorted(set(fetch) | set(write)):
        nf, vf = fetch.get(k, [0, 0.0])
        nw, vw = write.get(k, [0, 0.0])
        n = max(nf, nw, 1)
        out[k] = {"launches": n, "fetch_bytes_per_launch": vf / max(nf, 1),
                  "fetch_bytes_wide_corrected_per_launch": 2 * vf / max(nf, 1),
                  "write_bytes_per_launch": vw / max(nw, 1)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
