#!/bin/bash
# Round 4: wideband tests on the two-block analysis, then same-box A/B of the C3 step:
# one-block analysis (env), two-block at 5 waves/SIMD (product), two-block at 4 waves/SIMD (variant).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_wideband.py \
  tests/test_spectrum.py tests/test_scanner.py -m gpu > $O/r04c_pytest.log 2>&1 || rc=$?
tail -1 $O/r04c_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
AB_ARGS="--chain wideband --pipeline off" bash tools/ab.sh env "TETRA_WB_ANALYSIS=1" "TETRA_WB_ANALYSIS=2" > $O/r04c_ab_env.txt 2>&1
AB_ARGS="--chain wideband --pipeline off" bash tools/ab.sh run tetraear-bladerf_amd/lib/libtetra_hip.so \
  tetraear-bladerf_amd/lib/variants/libwb_a2_lb4.so > $O/r04c_ab_lb.txt 2>&1
AB_ARGS="--chain wideband" AB_ROUNDS=2 bash tools/ab.sh env "TETRA_WB_ANALYSIS=1" "TETRA_WB_ANALYSIS=2" > $O/r04c_ab_env_pipe.txt 2>&1
echo done
