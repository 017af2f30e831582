#!/bin/bash
# Round 6: the per-wave analysis kernel (TETRA_WB_ANALYSIS=5) -- wideband tests (every form, the
# one-block forms bit-identical, the random sweep), then the wideband bench with forms 1 and 5
# alternating, serial and pipelined.  usage: bash tools/r06_wb_analysis.sh [rounds]
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wideband.py tests/test_gpu_fuzz.py -k "wideband or channelize or analysis" -q --timeout 200 --timeout-method thread > $O/r06_pytest_wb.log 2>&1 || { rc=$?; tail -30 $O/r06_pytest_wb.log; exit $rc; }
tail -2 $O/r06_pytest_wb.log
for r in $(seq ${1:-3}); do
  for pipe in off on; do
    for f in 1 5; do
      TETRA_WB_ANALYSIS=$f timeout -k 10 300 python -u bench.py --no-cpu --chain wideband --pipeline $pipe > $O/r06_wb_ab.log 2>&1
      python - "$f" "$pipe" <<'PY'
import json, sys
l = [json.loads(x) for x in open('gpurun_out/r06_wb_ab.log') if x.startswith('{"metric')][-1]
print("form", sys.argv[1], "pipeline", sys.argv[2], l["ms_per_step"], l["stages_ms_per_step"], flush=True)
PY
    done
  done
done
