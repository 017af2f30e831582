#!/bin/bash
# Round 6 (build with tools/ab_patches/timing_lds_pad.diff applied): the wideband timing stage at the occupancy a resampler + timing kernel with
# a chunk's y in LDS would have -- TETRA_TIMING_LDS_PAD bytes of unused LDS per one-wave workgroup --
# serial (--pipeline off), then the default pipelined step.  usage: bash tools/r06_wb_pad.sh [rounds]
set -e
O=gpurun_out; mkdir -p $O
for r in $(seq ${1:-2}); do
  for pad in 0 26624 37888 59392; do
    TETRA_TIMING_LDS_PAD=$pad timeout -k 10 300 python -u bench.py --no-cpu --chain wideband --pipeline off > $O/r06_wb_pad.log 2>&1
    python - "$pad" <<'PY'
import json, sys
l = [json.loads(x) for x in open('gpurun_out/r06_wb_pad.log') if x.startswith('{"metric')][-1]
print("pad", sys.argv[1], "serial", l["ms_per_step"], l["stages_ms_per_step"], flush=True)
PY
  done
done
timeout -k 10 300 python -u bench.py --no-cpu --chain wideband > $O/r06_wb_pad.log 2>&1
python - <<'PY'
import json
l = [json.loads(x) for x in open('gpurun_out/r06_wb_pad.log') if x.startswith('{"metric')][-1]
print("default pipelined", l["ms_per_step"], l["stages_ms_per_step"], flush=True)
PY
