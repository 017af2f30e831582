#!/bin/bash
# SQ counters of the lower-MAC kernels (k_etsi_viterbi, k_etsi_sync) over a short serial bench run.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_etsi" --output-format csv -d $O/a -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --pipeline off > $O/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC --kernel-include-regex "k_etsi" --output-format csv -d $O/b -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --pipeline off > $O/b.log 2>&1
python3 - <<PY
import csv, glob, collections
for d in ("a", "b"):
    f = glob.glob("$O/%s/**/*counter_collection.csv" % d, recursive=True)
    if not f: print("no csv", d); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0][-40:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print(d, k, {c: round(x) for c, x in v.items()})
PY
