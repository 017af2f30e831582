# compat GPU suite, then the latency probe under the kernel trace
set -e
R=$GRAFT_REPO_ROOT; cd $R
rc=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_compat.py > gpurun_out/r05_compat_t5.log 2>&1 || rc=$?
tail -2 gpurun_out/r05_compat_t5.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probe_compat_latency.py > gpurun_out/r05_compat_latency_v7.log 2>&1
python3 -c "
import json; t=open('gpurun_out/r05_compat_latency_v7.log').read(); d=json.loads(t[t.index('{'):]); print({k:(v['wall_ms_median'], {s:x[0] for s,x in v['stages_ms'].items()}) for k,v in d.items()})"
bash tools/prof_compat_latency.sh
