#!/bin/bash
# Refill-policy sweep: one bench line per (extra args, worker count), each under its own time
# limit; stops at the first failure.
#   tools/retry_sweep.sh TAG "common args" "workers..." ["variant args" ...]
tag=$1; common=$2; workers=$3; shift 3
variants=("$@"); [ ${#variants[@]} -eq 0 ] && variants=("")
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
i=0
for v in "${variants[@]}"; do
  for w in $workers; do
    echo "v$i w$w: $common $v" >> $out/index.txt
    timeout -k 10 180 python bench.py $common $v --workers $w --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 \
      > $out/v${i}_w$w.log 2>&1 || exit 1
  done
  i=$((i+1))
done
