set -e
O=gpurun_out/var; mkdir -p $O
for v in "fused" "split" "split --pipeline off" "split --iq sc16 --pipeline on" "split --iq sc16 --pipeline off" "fused --iq sc16"; do
  n=$(echo $v | tr ' ' '_' | tr -d '-')
  timeout -k 10 200 python -u bench.py --no-cpu --demod $v > $O/$n.log 2>&1
  python -c "import json,sys; d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][-1]; print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms_per_step'])"
done
