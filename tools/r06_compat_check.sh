#!/bin/bash
# Round 6: the compat chain's default form on the GPU (tests + smoke + C2 latency), then its
# rocprof evidence (kernel trace + FETCH / WRITE PMC of bench.py --chain compat).
# usage: bash tools/r06_compat_check.sh [tests] [latency] [prof]
set -e
O=gpurun_out; mkdir -p $O
PARTS=${*:-tests latency prof}
for part in $PARTS; do
  case $part in
    tests)
      rc=0
      timeout -k 10 500 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_fuzz.py -k "compat or default or direct" -v --timeout 150 --timeout-method thread > $O/r06_pytest_compat.log 2>&1 || rc=$?
      tail -4 $O/r06_pytest_compat.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r06_smoke.log 2>&1
      tail -1 $O/r06_smoke.log ;;
    latency)
      timeout -k 10 300 python -u tools/latency_c2.py --reps 30 > $O/r06_c2_latency.log 2>&1
      cat $O/r06_c2_latency.log ;;
    prof)
      bash tools/profile_bench.sh ${PROFILE_COMPAT:-r06_compat_v1} --chain compat
      cat gpurun_out/prof/${PROFILE_COMPAT:-r06_compat_v1}/summary.log | head -30 ;;
  esac
done
