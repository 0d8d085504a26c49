#!/bin/bash
# Host-pointer boundary: the serving kernel's phases at 1 and 8 threads.   tools/gpu_hostprof.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out
for t in 1 8; do
  HKV_PART_PROF=1 HKV_HOST_TIMING=1 HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 2 50 > $out/prof$t.log 2>&1 || exit 5
done
