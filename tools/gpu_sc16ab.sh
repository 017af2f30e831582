#!/bin/bash
# ETSI GPU tests on the working library, then same-box SC16 A/B (pipelined, then serial) of the
# libraries in $AB
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_etsi.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_r.log 2>&1 || rc=$?
tail -3 $O/pt_r.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
AB_ARGS='--iq sc16' bash tools/ab_demod.sh $AB > $O/ab_sc16.txt 2>&1
AB_ARGS='--iq sc16 --pipeline off' bash tools/ab_demod.sh $AB > $O/ab_sc16s.txt 2>&1
echo done
