#!/bin/bash
# Round 6: SC16 stage 1 on the matrix cores (TETRA_SC16_S1=mfma) -- the ETSI GPU suites with it
# forced, then the SC16 bench, DPP and MFMA arms alternating on one box.
# usage: bash tools/r06_s1m.sh [rounds]
set -e
O=gpurun_out; mkdir -p $O
TETRA_SC16_S1=mfma timeout -k 10 600 python -u -m pytest tests/test_gpu_etsi.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py \
  -q -x --timeout 150 --timeout-method thread -k "etsi or stream or sc16 or SC16" > $O/r06_pytest_s1m.log 2>&1
tail -2 $O/r06_pytest_s1m.log
for r in $(seq ${1:-3}); do
  for arm in dpp mfma; do
    TETRA_SC16_S1=$arm timeout -k 10 300 python -u bench.py --no-cpu --iq sc16 > $O/r06_s1m_$arm.log 2>&1
    python - "$arm" <<'PY'
import json, sys
l = [json.loads(x) for x in open(f'gpurun_out/r06_s1m_{sys.argv[1]}.log') if x.startswith('{"metric')][-1]
print(sys.argv[1], l["ms_per_step"], l["roofline"]["launch_ms"], l["roofline"]["frac"], l["stages_ms_per_step"],
      l["decoded_last_step"].get("decoded_frac"), flush=True)
PY
  done
done
