#!/bin/bash
# Same-box A/B call: the ETSI GPU parity tests on the working library, then AB="libs..." pipelined cf32
# and SC16 (tools/ab_demod.sh, three rounds each).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_etsi.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_ab.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
AB_ARGS=" " bash tools/ab_demod.sh $AB > $O/ab_pipe.txt 2>&1
AB_ARGS="--iq sc16" bash tools/ab_demod.sh $AB > $O/ab_sc16.txt 2>&1
echo done
