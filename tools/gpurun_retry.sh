#!/bin/bash
# Retry a gpurun command while the pool reports a transient / no-box state
# (dev tool).  Usage: gpurun_retry.sh <timeout> <cmdfile> <outfile>
for i in $(seq 1 ${GPURUN_TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$(cat "$2")" > "$3" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$3"; then exit $rc; fi
  sleep 90
done
exit 3
