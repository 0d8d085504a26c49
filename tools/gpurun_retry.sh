#!/bin/bash
# usage: gpurun_retry.sh TIMEOUT "command"  -- retries only when gpurun reports no box/slot (rc 3)
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $1 -- "$2"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
