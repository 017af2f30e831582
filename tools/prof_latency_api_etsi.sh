set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof/r05_latency_api_etsi; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/tools/probes/latency_calls_etsi.py > $O/run.log 2>&1
tail -2 $O/run.log
python3 - <<PY
import csv, glob
for name in ("hip_api_stats", "kernel_stats"):
    f = glob.glob("$O/t/**/*%s.csv" % name, recursive=True)
    if not f: continue
    rows = list(csv.DictReader(open(f[0])))
    print("==", name)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 3), "ms total")
PY
