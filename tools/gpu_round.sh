#!/bin/bash
# GPU-box check: parity tests, smoke, default bench, wideband and SC16 benches; PROFILE=tag adds the
# rocprof passes of the default bench (tools/profile_bench.sh), PROFILE_SC16=tag those of the SC16 bench.  Every GPU step is time-limited and the steps
# are chained (set -e), so a fault or timeout ends the call.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
# test failures (rc 1) do not stop the call; anything else (a fault, a timeout, a crash) does
rc=0
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_etsi.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --cells given > $O/bench_etsi_given.log 2>&1
timeout -k 10 300 python -u bench.py --chain wideband --no-cpu > $O/bench_wb.log 2>&1
timeout -k 10 300 python -u bench.py --iq sc16 --no-cpu > $O/bench_sc16.log 2>&1
if [ -n "$PROFILE" ]; then bash tools/profile_bench.sh $PROFILE; fi
# PROFILE_SC16=tag: the same passes on the SC16 (BladeRF wire format) bench
if [ -n "$PROFILE_SC16" ]; then bash tools/profile_bench.sh $PROFILE_SC16 --iq sc16; fi
# AB="libA.so libB.so": same-box A/B of library variants, pipelined and serial cf32, pipelined SC16
if [ -n "$AB" ]; then
  AB_ARGS=" " bash tools/ab.sh run $AB > $O/ab_pipe.txt 2>&1
  if [ -n "$AB_SERIAL" ]; then AB_ARGS="--pipeline off" bash tools/ab.sh run $AB > $O/ab_serial.txt 2>&1; fi
  AB_ARGS="--iq sc16" bash tools/ab.sh run $AB > $O/ab_sc16.txt 2>&1
fi
echo done
