#!/bin/bash
# capi_threads at 8 / 16 threads under environment configurations, interleaved, 2 reps.  TAG CFG...
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
printf '%s\n' "$@" > $out/configs.txt
for rep in 1 2; do
  k=0
  for cfg in "$@"; do
    for t in 8 16; do
      env $cfg HKV_HOST_TIMING=1 HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/c${k}_t${t}_$rep.log 2>&1 || exit 12
    done
    k=$((k+1))
  done
done
exit 0
