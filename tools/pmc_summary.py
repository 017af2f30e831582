#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/<tag>_summary.json.

Inputs: a --kernel-trace --stats directory and separate --pmc FETCH_SIZE / WRITE_SIZE directories
(MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly
half of the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16-B/lane streaming stores and is taken as is).
usage: pmc_summary.py TRACE_DIR FETCH_DIR WRITE_DIR OUT_JSON [workload-string]
"""
import collections
import csv
import glob
import json
import sys


def _csv(d, name):
    f = glob.glob(f"{d}/**/*{name}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0].split("<")[0].replace("void ", "")


def main():
    trace, fetch, write, out = sys.argv[1:5]
    workload = sys.argv[5] if len(sys.argv) > 5 else ""
    stats = {short(r["Name"]): dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                    total_ns=float(r["TotalDurationNs"]), pct=float(r["Percentage"]))
             for r in _csv(trace, "kernel_stats.csv")}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in (fetch, write):
        for r in _csv(d, "counter_collection.csv"):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, s in stats.items():
        e = dict(s)
        if k in pmc:
            f = pmc[k].get("FETCH_SIZE", [])
            w = pmc[k].get("WRITE_SIZE", [])
            if f:
                e["fetch_size_kib_raw"] = sum(f) / len(f)
                e["read_bytes"] = 2 * 1024 * e["fetch_size_kib_raw"]   # gfx950 correction (x2)
            if w:
                e["write_size_kib"] = sum(w) / len(w)
                e["write_bytes"] = 1024 * e["write_size_kib"]
            if f and w:
                e["hbm_bytes_per_launch"] = e["read_bytes"] + e["write_bytes"]
        kernels[k] = e
    json.dump(dict(workload=workload, kernels=kernels), open(out, "w"), indent=1)
    print(json.dumps(kernels, indent=1)[:3000])


if __name__ == "__main__":
    main()
