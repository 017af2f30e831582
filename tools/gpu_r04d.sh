#!/bin/bash
# Round 4: the D = M / 2 one-block analysis (k_pfb_analysis1) and the timing ring: wideband + ETSI
# timing parity tests, then same-box A/B of the C3 step (serial and pipelined): ov2 one-block (new
# default), ov2 two-block, ov4 one-block (round 3), and the timing ring off.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_wideband.py \
  "tests/test_gpu_etsi.py::test_chanfilt_and_timing_bit_exact" "tests/test_gpu_etsi.py::test_timing_forms_bit_exact" "tests/test_gpu_etsi.py::test_fused_demod_many_channels" \
  "tests/test_gpu_etsi.py::test_demod_lengths_vs_oracle" tests/test_scanner.py \
  "tests/test_gpu_etsi.py::test_hard_symbol_decode_rate" -m gpu > $O/r04d_pytest.log 2>&1 || rc=$?
tail -1 $O/r04d_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
AB_ROUNDS=2 AB_ARGS="--chain wideband --pipeline off" bash tools/ab.sh env "TETRA_WB_OVERSAMPLE=2" "TETRA_WB_OVERSAMPLE=2 TETRA_WB_ANALYSIS=2" "TETRA_WB_OVERSAMPLE=2 TETRA_WB_ANALYSIS=3" \
  "TETRA_WB_OVERSAMPLE=4" "TETRA_WB_OVERSAMPLE=2 TETRA_TIMING_RING=2" "TETRA_WB_OVERSAMPLE=2 TETRA_TIMING_LEAN=0" "TETRA_WB_OVERSAMPLE=2 TETRA_WB_RESAMP_WT=1" > $O/r04d_ab_serial.txt 2>&1
AB_ROUNDS=2 AB_ARGS="--chain wideband" bash tools/ab.sh env "TETRA_WB_OVERSAMPLE=2" "TETRA_WB_OVERSAMPLE=2 TETRA_WB_ANALYSIS=2" "TETRA_WB_OVERSAMPLE=2 TETRA_WB_ANALYSIS=3" \
  "TETRA_WB_OVERSAMPLE=4" "TETRA_WB_OVERSAMPLE=2 TETRA_WB_RESAMP_WT=1" > $O/r04d_ab_pipe.txt 2>&1
AB_ARGS="--demod split" AB_ROUNDS=2 bash tools/ab.sh env "TETRA_TIMING_RING=1" "TETRA_TIMING_RING=2" "TETRA_TIMING_RING=1 TETRA_TIMING_LEAN=0" "TETRA_TIMING_RING=0" > $O/r04d_ab_split.txt 2>&1
echo done
