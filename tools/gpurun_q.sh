#!/bin/bash
# Queue a gpurun call: retries ONLY while gpurun answers "no box or slot free"
# (exit 3: nothing ran, nothing charged); any other outcome ends it.
# usage: tools/gpurun_q.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "nothing was charged" $OUT; then break; fi
  if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy\|no box\|no free box" $OUT; then break; fi
  sleep 90
done
echo "gpurun_q rc=$rc tries=$i" >> $OUT
