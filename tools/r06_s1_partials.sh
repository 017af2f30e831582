#!/bin/bash
# Round-6 A/B: stage 1 of k_chanfilt_r as block partials (five pk_fma chains per block, taps from
# LDS, four DPP-shifted adds per output) against the fma chain of round 5 (lib/variants/libs1old.so),
# SC16 and cf32, serial and the default pipelined step, same box, three rounds interleaved.
set -e
O=gpurun_out; mkdir -p $O
for a in "--iq sc16 --pipeline off" "--iq sc16" "--pipeline off" ""; do
  echo "== $a"
  AB_ARGS="$a" bash tools/ab.sh run tetraear-bladerf_amd/lib/libtetra_hip.so tetraear-bladerf_amd/lib/variants/libs1old.so
done
