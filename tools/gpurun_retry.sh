#!/bin/bash
# Submit one gpurun call; resubmit only while gpurun answers "no box / slot free" (exit 3, nothing ran,
# nothing charged), every 2 minutes, at most RETRIES (40) times.  Any other outcome (a result, a refusal, a
# failure of the command itself) ends it.  usage: tools/gpurun_retry.sh OUT TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for a in $(seq 1 ${RETRIES:-40}); do
  timeout $((TO + 1500)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  echo "EXIT $rc (attempt $a)" >> $OUT
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $OUT; then exit $rc; fi
  sleep 120
done
