#!/bin/bash
# Host-pointer boundary with the serving kernel: per-call timing, combining statistics and k_hserve's
# phases at 1 / 8 / 16 threads.   tools/gpu_hostprof.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out
for t in 1 8 16; do
  HKV_HOST_STATS=1 HKV_PART_PROF=1 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 \
    > $out/prof_t$t.log 2>&1 || exit 5
done
exit 0
