set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_etsi.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_prod.log 2>&1
tail -1 $O/pt_prod.log
TETRA_HIP_LIB=$R/tetraear-bladerf_amd/lib/variants/liblmac_v64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_etsi.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_v64.log 2>&1
tail -1 $O/pt_v64.log
AB_ARGS=" " bash tools/ab_demod.sh $AB > $O/ab_pipe.txt 2>&1
AB_ARGS="--pipeline off" bash tools/ab_demod.sh $AB > $O/ab_serial.txt 2>&1
AB_ARGS="--iq sc16" bash tools/ab_demod.sh $AB > $O/ab_sc16p.txt 2>&1
echo done
