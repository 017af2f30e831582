#!/bin/bash
# Round-6: the compat batch bench's step against its number of lanes (streams with a whole chain each),
# same box, three rounds interleaved.
set -e
O=gpurun_out; mkdir -p $O
for r in 1 2 3; do
  for n in 2 3 4; do
    timeout -k 10 200 python -u bench.py --chain compat --no-cpu --steps 30 --compat-lanes $n > $O/r06_lanes.log 2>&1
    python3 - "$r" "$n" <<'PY'
import json,sys
l=[json.loads(x) for x in open('gpurun_out/r06_lanes.log') if x.startswith('{"metric')][-1]
print("round", sys.argv[1], "lanes", sys.argv[2], l["ms_per_step"], l["value"], flush=True)
PY
  done
done
