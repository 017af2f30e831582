#!/bin/bash
# Full GPU suite + smoke, then the compat chain's rocprof passes (tools/profile_bench.sh) and bench
# lines.  Every GPU step is time-limited and chained.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/profile_bench.sh r03_compat_v1 --chain compat
cd $R
timeout -k 10 300 python -u bench.py --chain compat --no-cpu > $O/bench_compat.log 2>&1
timeout -k 10 300 python -u bench.py --chain compat --pipeline off --no-cpu > $O/bench_compat_serial.log 2>&1
echo done
