#!/usr/bin/env python3
"""Summarise rocprofv3 runs of bench.py into profiles/<tag>_summary.json.

Inputs: a --kernel-trace --stats directory and separate --pmc FETCH_SIZE / WRITE_SIZE directories of
the SAME bench command (MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reads exactly half of the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B/lane streaming stores and is taken as is).

--timed K keeps, per kernel, only its last K launches (bench.py's timed steps: every kernel of the
step is launched once per step, after the warm-up steps and before nothing else that kernel runs),
for the average duration (from kernel_trace.csv) and for the counters, so the summary describes the
timed region the bench line's launch_ms and frac come from -- not warm-up launches.
usage: pmc_summary.py TRACE_DIR FETCH_DIR WRITE_DIR OUT_JSON [workload] [--timed K]
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


def _order(r):
    for k in ("Dispatch_Id", "Correlation_Id", "Start_Timestamp"):
        if r.get(k, "") not in ("", None):
            return int(r[k])
    return 0


def main():
    args = [a for a in sys.argv[1:]]
    timed = None
    if "--timed" in args:
        i = args.index("--timed")
        timed = int(args[i + 1])
        del args[i:i + 2]
    trace, fetch, write, out = args[:4]
    workload = args[4] if len(args) > 4 else ""
    stats = {short(r["Name"]): dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                    total_ns=float(r["TotalDurationNs"]), pct=float(r["Percentage"]))
             for r in _csv(trace, "kernel_stats.csv")}
    # per-launch durations of the timed launches
    launches = collections.defaultdict(list)
    for r in sorted(_csv(trace, "kernel_trace.csv"), key=_order):
        launches[short(r["Kernel_Name"])].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in (fetch, write):
        for r in sorted(_csv(d, "counter_collection.csv"), key=_order):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, s in stats.items():
        e = dict(s)
        d = launches.get(k, [])
        if timed and len(d) >= timed:
            sel = d[-timed:]
            e.update(timed_launches=timed, timed_avg_ns=sum(sel) / timed, timed_min_ns=min(sel),
                     timed_max_ns=max(sel))
        if k in pmc:
            f = pmc[k].get("FETCH_SIZE", [])
            w = pmc[k].get("WRITE_SIZE", [])
            if timed:
                f, w = f[-timed:], w[-timed:]
            if f:
                e["fetch_size_kib_raw"] = sum(f) / len(f)
                e["read_bytes"] = 2 * 1024 * e["fetch_size_kib_raw"]   # gfx950 correction (x2)
            if w:
                e["write_size_kib"] = sum(w) / len(w)
                e["write_bytes"] = 1024 * e["write_size_kib"]
            if f and w:
                e["hbm_bytes_per_launch"] = e["read_bytes"] + e["write_bytes"]
                e["pmc_launches"] = min(len(f), len(w))
        kernels[k] = e
    json.dump(dict(workload=workload, timed_launches_per_kernel=timed, kernels=kernels), open(out, "w"), indent=1)
    print(json.dumps(kernels, indent=1)[:3000])


if __name__ == "__main__":
    main()
