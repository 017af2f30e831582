#!/bin/bash
# GPU tests $TESTS on the working library, then same-box A/B of $AB over the bench argument sets
# in $ABSETS (';'-separated), three rounds each (tools/ab_demod.sh).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_ab5.log 2>&1
  tail -1 $O/pt_ab5.log
fi
i=0
IFS=';' read -ra SETS <<< "$ABSETS"
for a in "${SETS[@]}"; do
  i=$((i+1))
  echo "# $a" > $O/ab5_$i.txt
  AB_ARGS="$a" bash tools/ab_demod.sh $AB >> $O/ab5_$i.txt 2>&1
done
echo done
