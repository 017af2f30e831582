# what bounds the banked compat decimator: the serial compat bench on timing-only variants
set -e
R=$GRAFT_REPO_ROOT; cd $R
L=tetraear-bladerf_amd/lib
AB_ROUNDS=2 AB_ARGS="--chain compat --pipeline off" bash tools/ab.sh run $L/libtetra_hip.so $L/variants/libcompat_fwd_nostore.so $L/variants/libcompat_noload.so $L/variants/libcompat_nomem.so > gpurun_out/r05_ab_compat_mem.txt 2>&1
cat gpurun_out/r05_ab_compat_mem.txt
