#!/bin/bash
# usage: gpurun_retry.sh TIMEOUT "command"  -- re-issues a gpurun call only when no GPU box or slot was free
# (rc 3, or a "transient" status that charged nothing); GPU scripts never exit with 3
for i in $(seq 1 20); do
  out=$(/usr/local/graft/bin/gpurun --timeout $1 -- "$2" 2>&1)
  rc=$?
  echo "$out"
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
