export HKV_HOST_STATS=1
for t in 1 2 4 8 16; do ./tools/capi_threads throughput $t 1.0 50; done 2>&1
