#!/bin/bash
# Round 4: the AFC gate and the scanner detector on the GPU.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread \
  tests/test_spectrum.py tests/test_scanner.py -m gpu > $O/r04b_pytest.log 2>&1 || rc=$?
tail -1 $O/r04b_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
echo done
