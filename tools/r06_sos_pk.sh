#!/bin/bash
# Round-6 A/B: the fp32 decimator biquad on packed VALU (v_pk_mul_f32 / v_pk_add_f32, 6 instructions
# per section tick instead of 9) against the library with the scalar form (lib/variants/liboldsos.so,
# compat_demod.hip at the previous commit): the GPU suite on the new library, C2's one-chunk latency
# and the compat batch bench, same box, interleaved.
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > $O/r06_pytest_gpu_sospk.log 2>&1
tail -1 $O/r06_pytest_gpu_sospk.log
for r in 1 2; do
  for L in tetraear-bladerf_amd/lib/libtetra_hip.so tetraear-bladerf_amd/lib/variants/liboldsos.so; do
    TETRA_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/latency_c2.py --reps 30 > $O/r06_c2_sospk.log 2>&1
    echo "round $r $(basename $L) $(tail -1 $O/r06_c2_sospk.log | cut -c1-400)"
  done
done
AB_ARGS="--chain compat" bash tools/ab.sh run tetraear-bladerf_amd/lib/libtetra_hip.so tetraear-bladerf_amd/lib/variants/liboldsos.so
AB_ARGS="--chain compat --pipeline off" bash tools/ab.sh run tetraear-bladerf_amd/lib/libtetra_hip.so tetraear-bladerf_amd/lib/variants/liboldsos.so
