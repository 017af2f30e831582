# compat decimator DPP hand-off: GPU compat suite on the new library, then the compat bench
# alternating the previous library (lib/variants/libcompat_old.so) and the new one, serial and pipelined
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/abc
rc=0
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py > gpurun_out/abc/tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> gpurun_out/abc/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
L=tetraear-bladerf_amd/lib
for i in 1 2; do
  for lib in variants/libcompat_old.so libtetra_hip.so; do
    n=$(basename $lib .so)
    TETRA_HIP_LIB=$R/$L/$lib timeout -k 10 200 python -u bench.py --chain compat --no-cpu > gpurun_out/abc/$n.pipe.$i.log 2>&1
    TETRA_HIP_LIB=$R/$L/$lib timeout -k 10 200 python -u bench.py --chain compat --no-cpu --pipeline off > gpurun_out/abc/$n.serial.$i.log 2>&1
  done
done
for f in gpurun_out/abc/lib*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$(basename $f .log)', d['ms_per_step'], d['stages_ms_per_step'])"; done
