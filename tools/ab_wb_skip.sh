set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/wbs
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --chain wideband --no-cpu > gpurun_out/wbs/full.$i.log 2>&1
  WB_SKIP=waterfall timeout -k 10 200 python -u tools/probes/wb_skip.py --chain wideband --no-cpu > gpurun_out/wbs/nowf.$i.log 2>&1
done
for f in gpurun_out/wbs/*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$(basename $f .log)', d['ms_per_step'], d['stages_ms_per_step'])"; done
