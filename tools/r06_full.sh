#!/bin/bash
# Round 6: the whole GPU suite + smoke, then the rocprof evidence of the default (streaming) etsi bench
# and the compat bench.  usage: bash tools/r06_full.sh [tests] [prof] [profsc16] [profwb]
set -e
O=gpurun_out; mkdir -p $O
for part in ${*:-tests prof}; do
  case $part in
    tests)
      rc=0
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/r06_pytest_gpu.log 2>&1 || rc=$?
      tail -5 $O/r06_pytest_gpu.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r06_smoke.log 2>&1
      tail -1 $O/r06_smoke.log ;;
    prof)
      bash tools/profile_bench.sh ${PROFILE:-r06_etsi_v1}
      bash tools/profile_bench.sh ${PROFILE_COMPAT:-r06_compat_v1} --chain compat ;;
    profsc16)
      bash tools/profile_bench.sh ${PROFILE_SC16:-r06_etsi_sc16_v1} --iq sc16 ;;
    profwb)
      bash tools/profile_bench.sh ${PROFILE_WB:-r06_wideband_v1} --chain wideband ;;
  esac
done
echo done
