"""tools/pmc_summary.py on synthetic rocprofv3 CSVs (CPU): kernels keyed by full name, timed launches
selected between bench.py's k_region_mark launches, the FETCH x2 correction at every load width
(calibrated: profiles/r05_fetch_calibration.json), and the fallback to the last K launches when a trace has no markers."""
import csv
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pmc_summary as P  # noqa: E402

K16 = "void (anonymous namespace)::k_chanfilt_r<HIP_vector_type<float, 4u>, true>(HIP_vector_type<float, 4u> const*, long, int, (anonymous namespace)::TimingOut)"
K16B = "void (anonymous namespace)::k_chanfilt_r<HIP_vector_type<unsigned int, 4u>, true>(HIP_vector_type<unsigned int, 4u> const*, long, int, (anonymous namespace)::TimingOut)"
K8 = "void (anonymous namespace)::k_pfb_resamp_fix<36, 25, 23, false, 0, true>(HIP_vector_type<float, 2u> const*, int, int, float const*, HIP_vector_type<float, 2u>*, int, HIP_vector_type<float, 4u>*, int)"
KJ = "(anonymous namespace)::k_etsi_viterbi((anonymous namespace)::Job const*, unsigned long long const*, int, signed char const*, int)"
MARK = "(anonymous namespace)::k_region_mark(int, int*)"


def test_load_widths():
    assert P.load_width(K16) == 16 and P.load_width(K16B) == 16 and P.load_width(K8) == 8
    assert P.load_width(KJ) is None
    assert P.load_width("void (anonymous namespace)::k_waterfall<0, false>(void const*, unsigned long)") == \
        P.WIDTH_OVERRIDE["k_waterfall"]
    assert P.short(K16) == "k_chanfilt_r" and P.short(MARK) == "k_region_mark"


def _write(d, name, rows, fields):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _run(tmp, launches, counters, marks=True):
    """launches: [(name, dur_ns)] in dispatch order; counters: {name: (fetch_kib, write_kib)}."""
    seq = ([(MARK, 10)] if marks else []) + launches[2:] + ([(MARK, 10)] if marks else [])
    seq = launches[:2] + seq   # two setup / warm-up launches before the first mark
    tr, st, fe, wr = [], {}, [], []
    t = 0
    for i, (n, dur) in enumerate(seq):
        tr.append({"Dispatch_Id": i + 1, "Kernel_Name": n, "Start_Timestamp": t, "End_Timestamp": t + dur})
        t += dur + 5
        s = st.setdefault(n, {"Name": n, "Calls": 0, "TotalDurationNs": 0})
        s["Calls"] += 1
        s["TotalDurationNs"] += dur
        if n in counters:
            fe.append({"Dispatch_Id": i + 1, "Kernel_Name": n, "Counter_Name": "FETCH_SIZE", "Counter_Value": counters[n][0]})
            wr.append({"Dispatch_Id": i + 1, "Kernel_Name": n, "Counter_Name": "WRITE_SIZE", "Counter_Value": counters[n][1]})
        if n == MARK:
            fe.append({"Dispatch_Id": i + 1, "Kernel_Name": n, "Counter_Name": "FETCH_SIZE", "Counter_Value": 0})
            wr.append({"Dispatch_Id": i + 1, "Kernel_Name": n, "Counter_Name": "WRITE_SIZE", "Counter_Value": 0})
    for s in st.values():
        s["AverageNs"] = s["TotalDurationNs"] / s["Calls"]
        s["Percentage"] = 1.0
    _write(os.path.join(tmp, "trace"), "run_kernel_trace.csv", tr, list(tr[0]))
    _write(os.path.join(tmp, "trace"), "run_kernel_stats.csv", list(st.values()),
           ["Name", "Calls", "AverageNs", "TotalDurationNs", "Percentage"])
    _write(os.path.join(tmp, "fetch"), "run_counter_collection.csv", fe, list(fe[0]))
    _write(os.path.join(tmp, "write"), "run_counter_collection.csv", wr, list(wr[0]))
    out = os.path.join(tmp, "s.json")
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), os.path.join(tmp, "trace"),
                    os.path.join(tmp, "fetch"), os.path.join(tmp, "write"), out, "wl", "--timed", "2"],
                   check=True, capture_output=True)
    return json.load(open(out))


def test_marker_window_full_names_and_corrections(tmp_path):
    # setup: two launches of the SC16 instantiation (same short name) before the first mark
    launches = [(K16B, 900), (K16B, 900), (K16, 1000), (K8, 100), (K16, 1200), (K8, 120), (KJ, 50)]
    d = _run(str(tmp_path), launches, {K16: (1000.0, 10.0), K16B: (5000.0, 0.0), K8: (300.0, 200.0), KJ: (4.0, 2.0)})
    assert d["selection"] == "markers"
    k = d["kernels"]
    assert set(k) == {K16, K16B, K8, KJ}                        # the marker itself is not listed
    assert k[K16]["timed_launches"] == 2 and k[K16]["timed_avg_ns"] == 1100
    assert "timed_launches" not in k[K16B]                       # setup only: nothing timed, not merged
    assert k[K16]["fetch_correction"] == 2 and k[K16]["read_bytes"] == 2 * 1024 * 1000
    assert k[K8]["fetch_correction"] == 2 and k[K8]["hbm_bytes_per_launch"] == 1024 * (2 * 300 + 200)
    assert k[KJ]["fetch_correction"] == 2
    assert k[K8]["load_bytes_per_lane"] == 8   # information only


def test_no_markers_falls_back_to_last_k(tmp_path):
    launches = [(K16, 500), (K16, 500), (K16, 1000), (K16, 1200)]
    d = _run(str(tmp_path), launches, {K16: (1000.0, 10.0)}, marks=False)
    assert d["selection"] == "last 2"
    assert d["kernels"][K16]["timed_launches"] == 2 and d["kernels"][K16]["timed_avg_ns"] == 1100


def test_bench_lookup_prefers_in_window_entry(tmp_path):
    """bench.traffic_from_profiles picks, among a short name's full-name entries, the one with timed
    launches."""
    sys.path.insert(0, REPO)
    import bench
    launches = [(K16B, 900), (K16B, 900), (K16, 1000), (K16, 1200)]
    d = _run(str(tmp_path), launches, {K16: (1000.0, 10.0), K16B: (5000.0, 0.0)})
    d["workload"] = "wl"
    prof = tmp_path / "profiles"
    prof.mkdir()
    json.dump(d, open(prof / "r09_y_summary.json", "w"))
    t = bench.traffic_from_profiles("k_chanfilt_r", "wl", profiles=str(prof))
    assert t["bytes"] == 1024 * (2 * 1000 + 10) and t["rocprof_avg_ms"] == 0.0011


def test_summaries_carry_source_provenance_and_bench_rejects_stale(tmp_path):
    """a summary names the hash of the source its kernels were built from, and
    bench.traffic_from_profiles cites it only while that source is unchanged -- else bytes None with
    the reason (no silent fallback to an older profile of other code)."""
    sys.path.insert(0, REPO)
    import bench
    src = P.kernel_source("k_chanfilt_r")
    assert src and src["file"] == "etsi_rx.hip" and len(src["sha256"]) == 64
    assert P.kernel_source("k_sos_fwd_bank")["file"] == "compat_demod.hip"
    assert P.kernel_source("no_such_kernel") is None
    launches = [(K16, 500), (K16, 500), (K16, 1000), (K16, 1200)]
    d = _run(str(tmp_path), launches, {K16: (1000.0, 10.0)})
    assert d["kernels"][K16]["source"] == src
    prof = tmp_path / "profiles"
    prof.mkdir()
    d["workload"] = "C5 shard: 8 channels x 4 cf32"
    json.dump(d, open(prof / "r09_x_summary.json", "w"))
    t = bench.traffic_from_profiles("k_chanfilt_r", "8 channels x 4 cf32", profiles=str(prof))
    assert t["bytes"] == 1024 * (2 * 1000 + 10) and t["source"] == "r09_x_summary.json"
    d["kernels"][K16]["source"] = dict(src, sha256="0" * 64)   # profiled on other code
    json.dump(d, open(prof / "r09_x_summary.json", "w"))
    t = bench.traffic_from_profiles("k_chanfilt_r", "8 channels x 4 cf32", profiles=str(prof))
    assert t["bytes"] is None and "other code" in t["reason"]
    t = bench.traffic_from_profiles("k_chanfilt_r", "no such workload", profiles=str(prof))
    assert t["bytes"] is None and "no rocprofv3" in t["reason"]
