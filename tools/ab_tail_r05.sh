set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/fetchcal
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fetchcal/f -o run -- $R/tools/probes/probe_fetch > $R/gpurun_out/fetchcal/f.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/fetchcal/w -o run -- $R/tools/probes/probe_fetch > $R/gpurun_out/fetchcal/w.log 2>&1
cd $R
L=tetraear-bladerf_amd/lib
V="$L/libtetra_hip.so $L/variants/libtail_div_mul.so $L/variants/libtail_sum1.so $L/variants/libtail_nointerp.so $L/variants/libtail_one_block.so"
AB_ROUNDS=2 AB_ARGS="--iq sc16 --pipeline off --cells given --chunks 1" bash tools/ab.sh run $V > gpurun_out/r05_ab_tail_sc16.txt 2>&1
AB_ROUNDS=2 AB_ARGS="--pipeline off --cells given --chunks 1" bash tools/ab.sh run $V > gpurun_out/r05_ab_tail_cf32.txt 2>&1
