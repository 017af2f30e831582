#!/bin/bash
# Where the fused demod's time goes: serial-step A/B of timing-only variants (outputs wrong) on one box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
V=tetraear-bladerf_amd/lib/variants
AB_ARGS="--pipeline off" bash tools/ab_demod.sh tetraear-bladerf_amd/lib/libtetra_hip.so $V/libskip_tail.so $V/libskip_mfma.so $V/libskip_stage1.so $V/libskip_tail_mfma.so > $O/decomp.txt 2>&1
echo done
