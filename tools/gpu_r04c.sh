#!/bin/bash
# Round 4: wideband tests (the D = M / 2 filter bank, two blocks per analysis iteration) and the AFC
# gate / scanner tests, then same-box A/B of the C3 step: filter-bank designs (TETRA_WB_OVERSAMPLE
# 2 = new default, 4 = round 3's) and, at oversample 4, the one-block analysis (TETRA_WB_ANALYSIS=1).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_wideband.py \
  tests/test_spectrum.py tests/test_scanner.py -m gpu > $O/r04c_pytest.log 2>&1 || rc=$?
tail -1 $O/r04c_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
rc=0
TETRA_WB_OVERSAMPLE=4 timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread \
  tests/test_wideband.py -m gpu > $O/r04c_pytest_ov4.log 2>&1 || rc=$?
tail -1 $O/r04c_pytest_ov4.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
AB_ARGS="--chain wideband --pipeline off" bash tools/ab.sh env "TETRA_WB_OVERSAMPLE=2" "TETRA_WB_OVERSAMPLE=4" \
  "TETRA_WB_OVERSAMPLE=4 TETRA_WB_ANALYSIS=1" > $O/r04c_ab_serial.txt 2>&1
AB_ARGS="--chain wideband" bash tools/ab.sh env "TETRA_WB_OVERSAMPLE=2" "TETRA_WB_OVERSAMPLE=4" \
  "TETRA_WB_OVERSAMPLE=4 TETRA_WB_ANALYSIS=1" > $O/r04c_ab_pipe.txt 2>&1
echo done
