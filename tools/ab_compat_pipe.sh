# the compat bench (pipelined, its default) alternating the previous library and the current one
set -e
R=$GRAFT_REPO_ROOT; cd $R
L=tetraear-bladerf_amd/lib
AB_ROUNDS=4 AB_ARGS="--chain compat" bash tools/ab.sh run $L/variants/libcompat_old.so $L/libtetra_hip.so > gpurun_out/r05_ab_compat_handoff_pipe.txt 2>&1
cat gpurun_out/r05_ab_compat_handoff_pipe.txt
