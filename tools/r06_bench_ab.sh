#!/bin/bash
# Round-6 A/B of the streaming bench step (same box, one call): the GPU stream tests, then bench.py
# variants; prints ms_per_step, the stage times and the decoded fraction of each.
# usage: bash tools/r06_bench_ab.sh "ENV=.. args" ...   (no argument: the default line)
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -q --timeout 150 --timeout-method thread > $O/r06_pytest_stream2.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
tail -3 $O/r06_pytest_stream2.log
[ $# -eq 0 ] && set -- ""
for v in "$@"; do
  [ -z "$v" ] && v="A=0"
  set -- $v
  envs=(); while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/r06_bench_ab.log 2>&1
  python - "$v" <<'PY'
import json,sys
l=[json.loads(x) for x in open('gpurun_out/r06_bench_ab.log') if x.startswith('{"metric')][-1]
print(sys.argv[1] or "default", l["ms_per_step"], l["stages_ms_per_step"], l.get("decoded_last_step",{}).get("decoded_frac"), flush=True)
PY
done
