#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root), all three passes on the
# driver's own command (bench.py --gpus 1 --steps 20 --warmup 5; --no-cpu: the CPU baseline runs
# after the timed region and starts worker processes, which must not run under the profiler):
#   1. --kernel-trace --stats (per-launch durations; the summary keeps the 20 timed launches),
#   2. separate --pmc FETCH_SIZE and WRITE_SIZE passes (MI355X_MICROARCH.md: one TCC counter group
#      per pass; KiB units; gfx950 FETCH_SIZE counts half of a wide streaming read -> x2),
#   3. tools/pmc_summary.py --timed 20 -> gpurun_out/prof/<tag>/<tag>_summary.json (copy into profiles/).
# usage: tools/profile_bench.sh TAG [extra bench args...]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py $ARGS > $O/trace_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py $ARGS > $O/pmc_write.log 2>&1
W=$(python3 -c "import json; print([json.loads(l) for l in open('$O/trace_bench.log') if l.startswith('{\"metric')][-1]['config']['workload'])")
python3 $R/tools/pmc_summary.py $O/trace $O/pmc_fetch $O/pmc_write $O/${TAG}_summary.json "$W" --timed 20 > $O/summary.log
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/${TAG}_kernel_stats.csv
