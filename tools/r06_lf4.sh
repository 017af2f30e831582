#!/bin/bash
# Round-6 A/B: filter_signal's lfilter with its four states on a quad of lanes (Lfilt4, default)
# against one lane per stream (TETRA_COMPAT_LF=1), both with the packed fp32 decimator biquad, and
# the library before both (lib/variants/liboldsos.so): the GPU suite (and the compat tests with the
# one-lane form), C2's one-chunk latency and the compat batch bench, same box, interleaved.
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > $O/r06_pytest_gpu_lf4.log 2>&1
tail -1 $O/r06_pytest_gpu_lf4.log
TETRA_COMPAT_LF=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_fuzz.py -k "compat or process or direct" -m gpu -q -x --timeout 150 --timeout-method thread > $O/r06_pytest_gpu_lf1.log 2>&1
tail -1 $O/r06_pytest_gpu_lf1.log
L0=tetraear-bladerf_amd/lib/libtetra_hip.so; L1=tetraear-bladerf_amd/lib/variants/liboldsos.so
for r in 1 2; do
  for v in "lf4 $L0 4" "lf1 $L0 1" "old $L1 1"; do
    set -- $v
    TETRA_COMPAT_LF=$3 TETRA_HIP_LIB=$PWD/$2 timeout -k 10 300 python -u tools/latency_c2.py --reps 30 > $O/r06_c2_lf.log 2>&1
    python3 - "$r" "$1" <<'PY'
import json,sys
d=[json.loads(l) for l in open('gpurun_out/r06_c2_lf.log') if l.startswith('{')][-1]
print("round", sys.argv[1], sys.argv[2], "compat_process_ms", d["compat_process_ms"], "blocked", d["compat_blocked_process_ms"], flush=True)
PY
  done
done
for a in "--chain compat" "--chain compat --pipeline off"; do
  AB_ARGS="$a" bash tools/ab.sh env "TETRA_COMPAT_LF=4" "TETRA_COMPAT_LF=1" "TETRA_HIP_LIB=$PWD/$L1"
done
