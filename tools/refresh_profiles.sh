#!/bin/bash
# Round profiles of the current code: rocprofv3 kernel stats + PMC traffic of the default (etsi) bench,
# then the bench lines of every chain.  usage: tools/refresh_profiles.sh TAG (e.g. r02_etsi_v5)
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
bash $R/tools/profile_bench.sh $TAG
cd $R
timeout -k 10 200 python -u bench.py > $O/${TAG}_bench.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --pipeline off > $O/${TAG}_bench_serial.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --iq sc16 > $O/${TAG}_bench_sc16.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --chain wideband > $O/${TAG}_bench_wideband.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --chain compat > $O/${TAG}_bench_compat.log 2>&1
echo done
