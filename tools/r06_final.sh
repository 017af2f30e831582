#!/bin/bash
# Round 6, final evidence on one box per call (run from the repo root on the GPU box):
#   tests   -- the whole GPU suite + smoke()
#   prof    -- rocprof kernel trace + FETCH/WRITE PMC of the default ETSI bench and of --chain compat
#   prof2   -- the same for --iq sc16 and --chain wideband
#   bench   -- the four bench lines (default ETSI with its CPU baseline, SC16, wideband, compat)
# Each new *_summary.json is copied into profiles/ on the box before the bench lines run, so their
# roofline.traffic reads this round's summaries of the current sources.
# usage: bash tools/r06_final.sh PART... [V=tag suffix, default v2]
set -e
O=gpurun_out; mkdir -p $O
V=${V:-v2}
cp_summ() { cp $O/prof/$1/$1_summary.json profiles/ && cp $O/prof/$1/$1_kernel_stats.csv profiles/; }
for part in "$@"; do
  case $part in
    tests)
      rc=0
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/r06_pytest_gpu_$V.log 2>&1 || rc=$?
      tail -3 $O/r06_pytest_gpu_$V.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r06_smoke_$V.log 2>&1
      tail -1 $O/r06_smoke_$V.log ;;
    prof)
      bash tools/profile_bench.sh r06_etsi_$V && cp_summ r06_etsi_$V
      bash tools/profile_bench.sh r06_compat_$V --chain compat && cp_summ r06_compat_$V ;;
    prof2)
      bash tools/profile_bench.sh r06_etsi_sc16_$V --iq sc16 && cp_summ r06_etsi_sc16_$V
      bash tools/profile_bench.sh r06_wideband_$V --chain wideband && cp_summ r06_wideband_$V ;;
    bench)
      for a in "etsi:" "sc16:--iq sc16 --no-cpu" "wb:--chain wideband" "compat:--chain compat --no-cpu"; do
        n=${a%%:*}; args=${a#*:}
        timeout -k 10 400 python -u bench.py $args > $O/r06_bench_${n}_$V.log 2>&1
        tail -1 $O/r06_bench_${n}_$V.log | cut -c1-400
      done ;;
  esac
done
echo done
