#!/bin/bash
# ETSI GPU tests on the working library, then same-box A/B of $AB: cf32 pipelined, cf32 serial, SC16 serial
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_etsi.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_ab3.log 2>&1 || rc=$?
[ -n "$NOTEST" ] || tail -2 $O/pt_ab3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
AB_ARGS=" " bash tools/ab_demod.sh $AB > $O/ab_pipe.txt 2>&1
AB_ARGS="--pipeline off" bash tools/ab_demod.sh $AB > $O/ab_serial.txt 2>&1
AB_ARGS="--iq sc16 --pipeline off" bash tools/ab_demod.sh $AB > $O/ab_sc16s.txt 2>&1
echo done
