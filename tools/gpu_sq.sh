#!/bin/bash
# SQ wave-cycle split of the fused demod (cf32 and SC16, serial bench) and the compat chain's bench
# lines (pipelined and serial).  Every GPU step is time-limited and chained (set -e).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/pmc_sq.sh r03_sq_cf32r
python3 tools/sq_summary.py $O/prof/r03_sq_cf32r/sq1 $O/prof/r03_sq_cf32r/sq2 $O/r03_sq_cf32r.json
bash tools/pmc_sq.sh r03_sq_sc16r2 --iq sc16
python3 tools/sq_summary.py $O/prof/r03_sq_sc16r2/sq1 $O/prof/r03_sq_sc16r2/sq2 $O/r03_sq_sc16r2.json
cd $R
timeout -k 10 300 python -u bench.py --chain compat --no-cpu > $O/bench_compat.log 2>&1
timeout -k 10 300 python -u bench.py --chain compat --pipeline off --no-cpu > $O/bench_compat_serial.log 2>&1
echo done
