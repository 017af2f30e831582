# leaf-parallel extract_symbols for every batch: GPU compat suite, then the compat bench (serial and
# pipelined) alternating the previous library (lib/variants/libextract_old.so) and the current one
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/exl
rc=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py > gpurun_out/exl/tests.log 2>&1 || rc=$?
tail -1 gpurun_out/exl/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
L=tetraear-bladerf_amd/lib
AB_ROUNDS=2 AB_ARGS="--chain compat --pipeline off" bash tools/ab.sh run $L/variants/libextract_old.so $L/libtetra_hip.so > gpurun_out/exl/serial.txt 2>&1
AB_ROUNDS=3 AB_ARGS="--chain compat" bash tools/ab.sh run $L/variants/libextract_old.so $L/libtetra_hip.so > gpurun_out/exl/pipe.txt 2>&1
cat gpurun_out/exl/serial.txt gpurun_out/exl/pipe.txt
