# per-kernel times of one-chunk compat process() calls (latency mode) under rocprofv3 --kernel-trace
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof/r05_compat_latency; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/probe_compat_latency.py > $O/probe.log 2>&1
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
