#!/bin/bash
# Same-box A/B of environment settings on the default (pipelined) bench:
#   tools/ab_env.sh "A=1" "A=0 B=2" ...   (3 rounds each)
set -e
O=gpurun_out/abenv; mkdir -p $O
for i in 1 2 3; do
  k=0
  for E in "$@"; do
    k=$((k+1))
    env $E timeout -k 10 200 python -u bench.py --no-cpu --steps 30 > $O/$k.$i.log 2>&1
    python -c "import json; d=[json.loads(l) for l in open('$O/$k.$i.log') if l.startswith('{')][-1]; print('$E', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
  done
done
