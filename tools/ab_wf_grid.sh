set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/wfg
for i in 1 2; do
  for g in 1024 512 256 128; do
    TETRA_WF_GRID=$g timeout -k 10 200 python -u bench.py --chain wideband --no-cpu > gpurun_out/wfg/g$g.$i.log 2>&1
  done
done
for f in gpurun_out/wfg/*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$(basename $f .log)', d['ms_per_step'], d['stages_ms_per_step'])"; done
