#!/bin/bash
# Round-end evidence on the final code, in parts that each fit one gpurun call:
#   tests  -- the GPU suite and smoke()
#   bench  -- the bench lines of every chain (default cf32 with cells acquired, cells given, SC16,
#             wideband, compat)
#   prof   -- the rocprof passes (kernel trace + FETCH / WRITE PMC) of the default, SC16 and wideband
#             benches (PROFILE, PROFILE_SC16, PROFILE_WB name them)
# usage: bash tools/gpu_final.sh [tests] [bench] [prof]   (no argument: all three)
# Every GPU step is time-limited and chained; test failures (rc 1) do not stop the call, anything else
# (a fault, a timeout, a crash) does.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
PARTS=${*:-tests bench prof}
for part in $PARTS; do
  case $part in
    tests)
      rc=0
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
      tail -1 $O/pytest_gpu.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      ;;
    bench)
      timeout -k 10 400 python -u bench.py > $O/bench_etsi.log 2>&1
      timeout -k 10 300 python -u bench.py --no-cpu --cells given > $O/bench_etsi_given.log 2>&1
      timeout -k 10 300 python -u bench.py --iq sc16 --no-cpu > $O/bench_sc16.log 2>&1
      timeout -k 10 300 python -u bench.py --chain wideband --no-cpu > $O/bench_wb.log 2>&1
      timeout -k 10 300 python -u bench.py --chain compat --no-cpu > $O/bench_compat.log 2>&1
      ;;
    prof)
      bash tools/profile_bench.sh ${PROFILE:-r04_etsi_v1}
      bash tools/profile_bench.sh ${PROFILE_SC16:-r04_etsi_sc16_v1} --iq sc16
      bash tools/profile_bench.sh ${PROFILE_WB:-r04_wideband_v1} --chain wideband
      ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
echo done
