set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/fetchcal
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fetchcal/f -o run -- $R/tools/probes/probe_fetch > $R/gpurun_out/fetchcal/f.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/fetchcal/w -o run -- $R/tools/probes/probe_fetch > $R/gpurun_out/fetchcal/w.log 2>&1
cd $R
rc=0
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py tests/test_scanner.py > gpurun_out/r05_t3.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/r05_t3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probe_compat_latency.py > gpurun_out/r05_compat_latency_v2.log 2>&1
L=tetraear-bladerf_amd/lib
V="$L/libtetra_hip.so $L/variants/libtail_div_mul.so $L/variants/libtail_sum1.so $L/variants/libtail_nointerp.so $L/variants/libtail_one_block.so $L/variants/libtail_specwin.so"
AB_ROUNDS=2 AB_ARGS="--iq sc16 --pipeline off --cells given --chunks 1" bash tools/ab.sh run $V > gpurun_out/r05_ab_tail_sc16.txt 2>&1
AB_ROUNDS=2 AB_ARGS="--pipeline off --cells given --chunks 1" bash tools/ab.sh run $V > gpurun_out/r05_ab_tail_cf32.txt 2>&1
rc=0
TETRA_HIP_LIB=$R/$L/variants/libtail_specwin.so timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_etsi.py -k "chanfilt_and_timing or fused_demod_many or demod_lengths or sc16_ingest or c5_full or every_cli_rate" > gpurun_out/r05_specwin_tests.log 2>&1 || rc=$?
echo "specwin pytest rc=$rc" >> gpurun_out/r05_specwin_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
