# the compat bench with the time-blocked decimator + filtfilt for the whole 8192-channel batch
# (TETRA_BENCH_COMPAT_DECIMATOR=blocked) against the default sequential passes, serial and pipelined
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/cbb
rc=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py > gpurun_out/cbb/tests.log 2>&1 || rc=$?
tail -1 gpurun_out/cbb/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for mode in serial pipe; do
    A=""; [ $mode = serial ] && A="--pipeline off"
    timeout -k 10 300 python -u bench.py --chain compat --no-cpu $A > gpurun_out/cbb/seq.$mode.$i.log 2>&1
    TETRA_BENCH_COMPAT_DECIMATOR=blocked timeout -k 10 300 python -u bench.py --chain compat --no-cpu $A > gpurun_out/cbb/blk.$mode.$i.log 2>&1
  done
done
for f in gpurun_out/cbb/*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$(basename $f .log)', d['ms_per_step'], d['stages_ms_per_step'], d.get('decoded_last_step'))"; done
