"""FETCH_SIZE / WRITE_SIZE calibration (tools/fetch_calib.hip under rocprofv3 --pmc, one pass per counter): for
each access pattern, the counter's bytes (FETCH_SIZE, WRITE_SIZE are in KiB) over the pattern's known bytes, per
kernel averaged over its launches. MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half of a 16-B-per-lane streaming
read on gfx950; this measures the factor for the engine's own access patterns (4-B and 8-B gathers, 4-B scatters).
usage: python tools/calib_summary.py <calib.json> <fetch_pass_dir> <write_pass_dir> <out.json>"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for x in csv.DictReader(open(f"{path}/run_counter_collection.csv")):
        if x["Counter_Name"] == counter:
            acc[x["Kernel_Name"].split("(")[0].replace("void ", "").strip()].append(float(x["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    truth = json.load(open(sys.argv[1]))
    fetch, write = per_kernel(sys.argv[2], "FETCH_SIZE"), per_kernel(sys.argv[3], "WRITE_SIZE")
    out = {}
    for k, t in truth.items():
        e = {"known": t}
        if "read" in t and k in fetch:
            e["fetch_size_bytes"] = fetch[k]
            e["fetch_over_read"] = round(fetch[k] / t["read"], 4)
            if "sectors" in t:
                e["fetch_per_sector"] = round(fetch[k] / t["sectors"], 2)
        if "write" in t and k in write:
            e["write_size_bytes"] = write[k]
            e["write_over_written"] = round(write[k] / t["write"], 4)
            if "sectors" in t:
                e["write_per_sector"] = round(write[k] / t["sectors"], 2)
        out[k] = e
    json.dump(out, open(sys.argv[4], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
