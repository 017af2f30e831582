#!/bin/bash
# Round-end evidence on the final code: GPU suite, smoke, the bench lines of every chain, and the
# rocprof passes of the default (cf32) and SC16 benches.  Every GPU step is time-limited, chained.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_etsi.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --cells acquire > $O/bench_etsi_acquire.log 2>&1
timeout -k 10 300 python -u bench.py --iq sc16 --no-cpu > $O/bench_sc16.log 2>&1
timeout -k 10 300 python -u bench.py --chain wideband --no-cpu > $O/bench_wb.log 2>&1
timeout -k 10 300 python -u bench.py --chain compat --no-cpu > $O/bench_compat.log 2>&1
bash tools/profile_bench.sh ${PROFILE:-r03_etsi_v5}
bash tools/profile_bench.sh ${PROFILE_SC16:-r03_etsi_sc16_v3} --iq sc16
echo done
