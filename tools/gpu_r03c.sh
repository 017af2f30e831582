set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 1 ] || exit $rc; }
tail -2 gpurun_out/pytest_gpu.log
NOTEST=1 AB='tetraear-bladerf_amd/lib/variants/libhead.so tetraear-bladerf_amd/lib/libtetra_hip.so' AB2='tetraear-bladerf_amd/lib/variants/libhead.so tetraear-bladerf_amd/lib/libtetra_hip.so' bash tools/gpu_ab2.sh
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log
