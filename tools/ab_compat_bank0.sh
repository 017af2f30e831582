# the banked decimator with bank-0 lanes loading their own samples (one DPP move per tick) against
# the product: serial compat bench, then the pipelined default
set -e
R=$GRAFT_REPO_ROOT; cd $R
L=tetraear-bladerf_amd/lib
AB_ROUNDS=3 AB_ARGS="--chain compat --pipeline off" bash tools/ab.sh run $L/libtetra_hip.so $L/variants/libcompat_bank0.so > gpurun_out/r05_ab_compat_bank0_serial.txt 2>&1
AB_ROUNDS=3 AB_ARGS="--chain compat" bash tools/ab.sh run $L/libtetra_hip.so $L/variants/libcompat_bank0.so > gpurun_out/r05_ab_compat_bank0_pipe.txt 2>&1
cat gpurun_out/r05_ab_compat_bank0_*.txt
