#!/bin/bash
# Round 4, first GPU call: the new C5 / streaming-acquire / RCCL / per-block MAC tests, then the
# default bench and the acquire bench (8 rotating chunks) on the same box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_etsi.py::test_c5_full_shard_8192x131072 tests/test_gpu_etsi.py::test_acquire_streaming_chunks \
  tests/test_gpu_etsi.py::test_etsi_frames_mac_per_block tests/test_gpu_etsi.py::test_process_and_decode_surface \
  tests/test_gpu_etsi.py::test_every_cli_rate_vs_oracle_and_round_trip \
  tests/test_gpu_etsi.py::test_generic_kernel_equals_fused_at_2400k \
  tests/test_gpu_etsi.py::test_unsupported_rate_never_raises_into_the_loop \
  tests/test_gpu_dist.py > $O/r04a_pytest.log 2>&1 || rc=$?
tail -1 $O/r04a_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu > $O/r04a_bench_given.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --cells acquire > $O/r04a_bench_acquire.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > $O/r04a_bench_given2.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --cells acquire > $O/r04a_bench_acquire2.log 2>&1
echo done
