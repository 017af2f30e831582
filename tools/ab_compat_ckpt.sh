# checkpointed compat decimator: GPU compat suite, then the compat bench (serial and pipelined)
# alternating the banked pair (TETRA_COMPAT_CKPT=0), the checkpointed pair, and the same built
# without SLP vectorisation
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/ck
rc=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py > gpurun_out/ck/tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/ck/tests.log
tail -3 gpurun_out/ck/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
L=tetraear-bladerf_amd/lib
for i in 1 2; do
  for mode in serial pipe; do
    A=""; [ $mode = serial ] && A="--pipeline off"
    TETRA_COMPAT_CKPT=0 timeout -k 10 200 python -u bench.py --chain compat --no-cpu $A > gpurun_out/ck/bank.$mode.$i.log 2>&1
    timeout -k 10 200 python -u bench.py --chain compat --no-cpu $A > gpurun_out/ck/ckpt.$mode.$i.log 2>&1
    TETRA_HIP_LIB=$R/$L/variants/libcompat_noslp.so timeout -k 10 200 python -u bench.py --chain compat --no-cpu $A > gpurun_out/ck/noslp.$mode.$i.log 2>&1
  done
done
for f in gpurun_out/ck/*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{\"metric'):
        d=json.loads(l); s=d['stages_ms_per_step']; print('$(basename $f .log)', d['ms_per_step'], s['compat_sos_fwd'], s['compat_sos_bwd'], d['decoded_last_step'] if 'decoded_last_step' in d else '')"; done
