set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/abwb
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --chain wideband --no-cpu > gpurun_out/abwb/cur.$i.log 2>&1
  (cd abtree_r04 && timeout -k 10 200 python -u bench.py --chain wideband --no-cpu > ../gpurun_out/abwb/r04.$i.log 2>&1)
done
for f in gpurun_out/abwb/*.log; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$f', d['ms_per_step'], d['stages_ms_per_step'])"; done
