#!/bin/bash
# Round 4, late: the F3 analysis (fold on three waves, select-base indexing, stage 2's last butterflies
# on the loader) against the fold-in-radix-8 form, and the timing ring in the pipelined wideband step
# (the ring's 4 KB of LDS per wave cannot co-reside with the channeliser's workgroups).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_wideband.py -m gpu \
  -k "analysis or timing_bit_exact or pipeline" > $O/r04r_pytest.log 2>&1 || rc=$?
tail -1 $O/r04r_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
AB_ROUNDS=2 AB_ARGS="--chain wideband --pipeline off" bash tools/ab.sh env "TETRA_WB_ANALYSIS=1" "TETRA_WB_ANALYSIS=4" "TETRA_WB_RESAMP_PROBE=1" > $O/r04r_ab_serial.txt 2>&1
AB_ROUNDS=3 AB_ARGS="--chain wideband" bash tools/ab.sh env "TETRA_TIMING_RING=1" "TETRA_TIMING_RING=0" > $O/r04r_ab_pipe.txt 2>&1
cut -c1-220 $O/r04r_ab_serial.txt $O/r04r_ab_pipe.txt
