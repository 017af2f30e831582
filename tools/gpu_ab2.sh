#!/bin/bash
# A/B call: ETSI + wideband GPU parity tests on the working library, then pipelined cf32 and serial cf32 A/B.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_etsi.py tests/test_wideband.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_ab.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
AB_ARGS=" " bash tools/ab_demod.sh $AB > $O/ab_pipe.txt 2>&1
if [ -n "$AB2" ]; then AB_ARGS="--pipeline off" bash tools/ab_demod.sh $AB2 > $O/ab_serial.txt 2>&1; fi
echo done
