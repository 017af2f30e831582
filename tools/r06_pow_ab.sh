#!/bin/bash
set -e
O=gpurun_out; mkdir -p $O
for r in 1 2; do
  for pipe in off on; do
    for v in 0 1 2; do
      TETRA_COMPAT_POW=$v timeout -k 10 300 python -u bench.py --no-cpu --chain compat --pipeline $pipe > $O/r06_pow.log 2>&1
      python - "$v" "$pipe" <<'PY'
import json, sys
l = [json.loads(x) for x in open('gpurun_out/r06_pow.log') if x.startswith('{"metric')][-1]
print("pow", sys.argv[1], "pipeline", sys.argv[2], l["ms_per_step"], l["stages_ms_per_step"], flush=True)
PY
    done
  done
done
