set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
rc=0
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/warm_probe.sh > $O/warm_probe.txt 2>&1
bash tools/profile_bench.sh r03_etsi_v2
timeout -k 10 300 python -u bench.py > $O/bench_etsi.log 2>&1
timeout -k 10 300 python -u bench.py --iq sc16 --no-cpu > $O/bench_sc16.log 2>&1
echo done
