#!/bin/bash
# SQ counters per kernel over a short serial bench run: tools/pmc_kernels.sh TAG REGEX [bench args]
set -e
TAG=$1; RX=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "$RX" --output-format csv -d $O/a -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu "$@" > $O/a.log 2>&1
python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/a/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    wc = v.get("SQ_WAVE_CYCLES", 1) or 1
    print(k, {c: round(x) for c, x in v.items()}, "wait_any %.2f wait_inst %.2f valu %.2f" % (v.get("SQ_WAIT_ANY",0)/wc, v.get("SQ_WAIT_INST_ANY",0)/wc, v.get("SQ_ACTIVE_INST_VALU",0)/wc))
PY
