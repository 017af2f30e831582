#!/bin/bash
# One-pass same-box A/B of library variants: tools/ab_once.sh lib1.so lib2.so ... (bench args from
# AB_ARGS, default the serial bench)
set -e
O=gpurun_out/ab; mkdir -p $O
for L in "$@"; do
  n=$(basename $L .so)
  TETRA_HIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-cpu --steps 20 ${AB_ARGS:---pipeline off} > $O/$n.log 2>&1
  python -c "import json; d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][-1]; print('$n', d['ms_per_step'], d['stages_ms_per_step'], d['roofline'].get('measured_read_floor_GBs'))"
done
