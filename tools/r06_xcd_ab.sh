#!/bin/bash
# Round-6 A/B: the C3 resampler's workgroups in XCD order (TETRA_WB_RESAMP_XCD=1) against dealt
# round-robin (0), same box, one call: the wideband tests with it, then three rounds of the pipelined
# and the serial bench step per arm, then one rocprof pass set per arm (FETCH / WRITE per kernel).
set -e
O=gpurun_out; mkdir -p $O
TETRA_WB_RESAMP_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_wideband.py -q -m gpu --timeout 150 --timeout-method thread > $O/r06_xcd_tests.log 2>&1
tail -1 $O/r06_xcd_tests.log
for r in 1 2 3; do
  for x in 0 1; do
    for p in "" "--no-pipeline"; do
      TETRA_WB_RESAMP_XCD=$x timeout -k 10 200 python -u bench.py --chain wideband --no-cpu $p > $O/r06_xcd_b.log 2>&1
      python3 - "$r" "$x" "$p" <<'PY'
import json,sys
l=[json.loads(x) for x in open('gpurun_out/r06_xcd_b.log') if x.startswith('{"metric')][-1]
print("round", sys.argv[1], "xcd", sys.argv[2], sys.argv[3] or "pipelined", l["ms_per_step"], l["stages_ms_per_step"], flush=True)
PY
    done
  done
done
for x in 0 1; do
  TETRA_WB_RESAMP_XCD=$x bash tools/profile_bench.sh r06_ab_xcd$x --chain wideband --no-pipeline
  python3 - $x <<'PY'
import json,sys
d=json.load(open(f'gpurun_out/prof/r06_ab_xcd{sys.argv[1]}/r06_ab_xcd{sys.argv[1]}_summary.json'))
for k,v in d['kernels'].items():
    if v.get('short') in ('k_pfb_resamp_fix','k_pfb_analysis1','k_timing'):
        print("xcd", sys.argv[1], v['short'], round(v['timed_avg_ns']/1e3,1), "us read", round(v['read_bytes']/1e6,1), "MB write", round(v['write_bytes']/1e6,1), "MB", flush=True)
PY
done
