#!/usr/bin/env python3
"""Summarise rocprofv3 runs of bench.py into profiles/<tag>_summary.json.

Inputs: a --kernel-trace --stats directory and separate --pmc FETCH_SIZE / WRITE_SIZE directories of
the SAME bench command.

* Kernels are keyed by their FULL demangled name (template arguments and signature), so two
  instantiations of one template -- or a kernel that only runs in setup -- never merge; each entry
  also carries its short name (``short``), which bench.py's roofline lookup matches.
* Timed launches: bench.py brackets its timed steps with two ``k_region_mark`` launches
  (``tetra_mark``); every dispatch between the first two marks, by dispatch id, is a timed launch.
  Kernels with no launch in that window (setup, warm-up only, the CPU baseline) get no ``timed_*``
  fields.  A trace without marks (older bench) falls back to ``--timed K``: each kernel's last K
  launches.
* HBM bytes (MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE / WRITE_SIZE are KiB.  On gfx950
  FETCH_SIZE reports exactly half the bytes of a coalesced streaming read, so read bytes are
  2 x FETCH_SIZE for every kernel; WRITE_SIZE is taken as is.  The guide states the half for 16-B
  loads; tools/probes/probe_fetch.hip measured it for 4-, 8- and 16-B loads alike (1 GiB read:
  FETCH_SIZE 0.500 of the bytes at each width; 512 MiB written: WRITE_SIZE 1.000;
  profiles/r05_fetch_calibration.json).  ``load_bytes_per_lane`` (the first pointer argument's
  element size, read from the demangled signature; ``void const*`` inputs from WIDTH_OVERRIDE) is
  kept as information only.
usage: pmc_summary.py TRACE_DIR FETCH_DIR WRITE_DIR OUT_JSON [workload] [--timed K]
"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys

MARK = "k_region_mark"
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tetraear-bladerf_amd", "csrc")


def kernel_source(short_name, csrc=CSRC):
    """Provenance of a kernel's code: {"file": <csrc file defining it>, "sha256": <hash of that file
    and common.h>} or None.  pmc_summary records it per kernel; bench.py accepts a summary's bytes
    only while the kernel's source still hashes the same, so a summary of older code is never cited
    (VERDICT r5 item 4).  No git needed: the GPU box gets the tree without .git."""
    pat = re.compile(r"\bvoid\s+" + re.escape(short_name) + r"\s*\(")
    common = os.path.join(csrc, "common.h")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip"))):
        text = open(f, "rb").read()
        if pat.search(text.decode("utf-8", "replace")):
            h = hashlib.sha256(text)
            if os.path.isfile(common):
                h.update(open(common, "rb").read())
            return {"file": os.path.basename(f), "sha256": h.hexdigest()}
    return None
FETCH_CORRECTION = 2   # calibrated at 4, 8 and 16 B per lane (docstring)
# kernels that take their streamed input as `const void *`: element bytes per lane load
WIDTH_OVERRIDE = {"k_waterfall": 8, "k_chanfilt_g": 8}
_SCALAR = {"float": 4, "int": 4, "unsigned int": 4, "double": 8, "long": 8, "unsigned long": 8, "short": 2,
           "unsigned short": 2, "char": 1, "signed char": 1, "unsigned char": 1, "__half": 2}


def _csv(d, name):
    f = glob.glob(f"{d}/**/*{name}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0].split("<")[0].replace("void ", "").strip()


def load_width(name):
    """Bytes per lane of the kernel's first pointer argument (None if it cannot be read)."""
    s = short(name)
    if s in WIDTH_OVERRIDE:
        return WIDTH_OVERRIDE[s]
    i = name.rfind(")")
    if i < 0:
        return None
    depth, j = 0, i
    while j >= 0:   # the '(' that opens the argument list
        depth += {")": 1, "(": -1}.get(name[j], 0)
        if depth == 0:
            break
        j -= 1
    if j < 0:
        return None
    depth, arg = 0, ""
    for ch in name[j + 1:i]:
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            depth -= 1
        if ch == "," and depth == 0:
            if "*" in arg:
                break
            arg = ""
            continue
        arg += ch
    if "*" not in arg:
        return None
    arg = arg.replace("const", "").replace("*", "").replace("__restrict__", "").strip()
    m = re.match(r"HIP_vector_type<(.+?),\s*(\d+)u?>", arg)
    if m:
        return _SCALAR.get(m.group(1).strip(), 0) * int(m.group(2)) or None
    return _SCALAR.get(arg)


def _order(r):
    for k in ("Dispatch_Id", "Correlation_Id", "Start_Timestamp"):
        if r.get(k, "") not in ("", None):
            return int(r[k])
    return 0


def window(rows, name_key):
    """(first, last) dispatch ids strictly inside the first two marker launches, or None."""
    marks = sorted(_order(r) for r in rows if short(r[name_key]) == MARK)
    return (marks[0], marks[1]) if len(marks) >= 2 else None


def main():
    args = list(sys.argv[1:])
    timed = None
    if "--timed" in args:
        i = args.index("--timed")
        timed = int(args[i + 1])
        del args[i:i + 2]
    trace, fetch, write, out = args[:4]
    workload = args[4] if len(args) > 4 else ""
    stats = {r["Name"]: dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                             total_ns=float(r["TotalDurationNs"]), pct=float(r["Percentage"]))
             for r in _csv(trace, "kernel_stats.csv")}
    rows = sorted(_csv(trace, "kernel_trace.csv"), key=_order)
    win = window(rows, "Kernel_Name")
    launches = collections.defaultdict(list)   # (dispatch id, duration) per full name
    for r in rows:
        launches[r["Kernel_Name"]].append((_order(r), float(r["End_Timestamp"]) - float(r["Start_Timestamp"])))

    def in_window(seq, w):
        if w is not None:
            return [x for x in seq if w[0] < x[0] < w[1]]
        return seq[-timed:] if timed and len(seq) >= timed else []

    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    pmc_win = {}
    for d in (fetch, write):
        crow = sorted(_csv(d, "counter_collection.csv"), key=_order)
        pmc_win[d] = window(crow, "Kernel_Name")
        for r in crow:
            pmc[r["Kernel_Name"]][(d, r["Counter_Name"])].append((_order(r), float(r["Counter_Value"])))
    kernels = {}
    for k, s in stats.items():
        if short(k) == MARK:
            continue
        e = dict(s, short=short(k))
        sel = in_window(launches.get(k, []), win)
        if sel:
            dur = [x[1] for x in sel]
            e.update(timed_launches=len(sel), timed_avg_ns=sum(dur) / len(dur), timed_min_ns=min(dur),
                     timed_max_ns=max(dur))
        wdt = load_width(k)
        e["load_bytes_per_lane"] = wdt
        src = kernel_source(e["short"])
        if src:
            e["source"] = src
        if k in pmc:
            f = [v for _, v in in_window(pmc[k].get((fetch, "FETCH_SIZE"), []), pmc_win[fetch])]
            w = [v for _, v in in_window(pmc[k].get((write, "WRITE_SIZE"), []), pmc_win[write])]
            if f:
                corr = FETCH_CORRECTION
                e["fetch_size_kib_raw"] = sum(f) / len(f)
                e["fetch_correction"] = corr
                e["read_bytes"] = corr * 1024 * e["fetch_size_kib_raw"]
            if w:
                e["write_size_kib"] = sum(w) / len(w)
                e["write_bytes"] = 1024 * e["write_size_kib"]
            if f and w:
                e["hbm_bytes_per_launch"] = e["read_bytes"] + e["write_bytes"]
                e["pmc_launches"] = min(len(f), len(w))
        kernels[k] = e
    json.dump(dict(workload=workload, selection="markers" if win else (f"last {timed}" if timed else "none"),
                   timed_launches_per_kernel=timed, kernels=kernels), open(out, "w"), indent=1)
    print(json.dumps({v["short"] + (" *" if "timed_launches" in v else ""): v.get("hbm_bytes_per_launch")
                      for v in kernels.values()}, indent=1)[:3000])


if __name__ == "__main__":
    main()
