set -e
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 120 python -u bench.py --no-cpu > gpurun_out/ab_fused_$i.log 2>&1
timeout -k 10 120 python -u bench.py --no-cpu --demod split > gpurun_out/ab_split_$i.log 2>&1
timeout -k 10 120 python -u bench.py --no-cpu --demod split --no-pipeline > gpurun_out/ab_split_serial_$i.log 2>&1
done
echo done
