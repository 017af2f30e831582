set -e
R=$GRAFT_REPO_ROOT; cd $R
rc=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py > gpurun_out/r05_compat_t6.log 2>&1 || rc=$?
tail -1 gpurun_out/r05_compat_t6.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/prof_compat_latency.sh | grep -E "scan|extract_lat|sosb|lfb"
timeout -k 10 200 python -u tools/latency_c2.py > gpurun_out/r05_c2_v2.log 2>&1 && tail -1 gpurun_out/r05_c2_v2.log
