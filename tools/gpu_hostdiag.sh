#!/bin/bash
# Host-pointer boundary diagnostics: tools/capi_threads throughput at 1/2/4/8/16 threads with the
# combining statistics and k_small phase timings.   tools/gpu_hostdiag.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out
for t in 1 2 4 8 16; do
  HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 2 50 > $out/host_t$t.log 2>&1 || exit 5
done
HKV_SMALL_PROF=64 HKV_PART_PROF=64 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput 8 2 50 > $out/host_prof8.log 2>&1 || exit 6
HKV_SMALL_PROF=64 HKV_PART_PROF=64 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput 1 2 50 > $out/host_prof1.log 2>&1 || exit 6
exit 0
