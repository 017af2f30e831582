# the whole GPU suite (staging touches every host-argument entry point), then the latency probe
set -e
R=$GRAFT_REPO_ROOT; cd $R
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r05_pytest_gpu_full_v3.log 2>&1 || rc=$?
tail -2 gpurun_out/r05_pytest_gpu_full_v3.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probe_compat_latency.py > gpurun_out/r05_compat_latency_v9.log 2>&1
python3 -c "
import json; t=open('gpurun_out/r05_compat_latency_v9.log').read(); d=json.loads(t[t.index('{'):]); print({k:(v['wall_ms_median'], {s:x[0] for s,x in v['stages_ms'].items()}) for k,v in d.items()})"
timeout -k 10 200 python -u tools/latency_c2.py > gpurun_out/r05_c2_v2.log 2>&1 || true
tail -1 gpurun_out/r05_c2_v2.log
