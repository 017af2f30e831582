# same-box A/B of library variants on the one-chunk compat latency probe (tools/probe_compat_latency.py):
# wall median and per-stage device ms of the automatic (latency) mode, AB_ROUNDS rounds interleaved
#   usage (GPU box): bash tools/ab_latency.sh LIB...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/ablat; mkdir -p $O
for i in $(seq 1 ${AB_ROUNDS:-3}); do
    for L in "$@"; do
        n=$(basename $L .so)
        TETRA_HIP_LIB=$R/$L timeout -k 10 200 python -u tools/probe_compat_latency.py > $O/$n.$i.log 2>&1
        python3 -c "
import json,sys; t=open(sys.argv[2]).read(); d=json.loads(t[t.index('{'):])['auto']
print(sys.argv[1], d['wall_ms_median'], {s: x[0] for s, x in d['stages_ms'].items()})" $n $O/$n.$i.log
    done
done
