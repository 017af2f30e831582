#!/bin/bash
# SQ + TA/TD counters of the compat decimator kernels over a short bench run: tools/pmc_compat.sh TAG
set -e
TAG=${1:-c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_compat_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "k_sos|k_lf" --output-format csv -d $O/a -o run -- python3 $R/bench.py --chain compat --steps 2 --warmup 1 --no-cpu > $O/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --kernel-include-regex "k_sos|k_lf" --output-format csv -d $O/b -o run -- python3 $R/bench.py --chain compat --steps 2 --warmup 1 --no-cpu > $O/b.log 2>&1 || echo "pass b failed"
python3 - <<PY
import csv, glob, collections
for d in ("a", "b"):
    f = glob.glob("$O/%s/**/*counter_collection.csv" % d, recursive=True)
    if not f: print("no csv", d); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        wc = v.get("SQ_WAVE_CYCLES", 0)
        extra = ""
        if wc:
            extra = "wait_any %.2f wait_inst %.2f valu %.2f" % (v.get("SQ_WAIT_ANY",0)/wc, v.get("SQ_WAIT_INST_ANY",0)/wc, v.get("SQ_ACTIVE_INST_VALU",0)/wc)
        print(d, k, {c: round(x) for c, x in v.items()}, extra)
PY
