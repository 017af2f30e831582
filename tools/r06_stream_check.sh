#!/bin/bash
# Round 6: the streaming ETSI receiver and the compat default on the GPU (tests), then a bench line.
# usage: bash tools/r06_stream_check.sh [tests] [bench] [prof TAG]
set -e
O=gpurun_out; mkdir -p $O
case ${1:-tests} in
  tests)
    rc=0
    timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_compat.py tests/test_gpu_fuzz.py -k "stream or compat or default or direct" -v --timeout 150 --timeout-method thread > $O/r06_pytest_stream.log 2>&1 || rc=$?
    tail -15 $O/r06_pytest_stream.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r06_smoke.log 2>&1
    tail -1 $O/r06_smoke.log ;;
  bench)
    shift
    timeout -k 10 400 python -u bench.py --no-cpu "$@" > $O/r06_bench_stream.log 2>&1
    tail -c 3000 $O/r06_bench_stream.log ;;
esac
