#!/bin/bash
# Does the bench's step time depend on how long the GPU has been busy?  The default bench three
# times back to back, then once with a long warm-up (untimed steps).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/warm; mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu > $O/default.$i.log 2>&1
  python -c "import json; d=[json.loads(l) for l in open('$O/default.$i.log') if l.startswith('{')][-1]; print('default', $i, d['ms_per_step'], d['roofline']['launch_ms'])"
done
timeout -k 10 200 python -u bench.py --no-cpu --warmup 300 > $O/warm300.log 2>&1
python -c "import json; d=[json.loads(l) for l in open('$O/warm300.log') if l.startswith('{')][-1]; print('warmup300', d['ms_per_step'], d['roofline']['launch_ms'])"
