#!/bin/bash
# Host entry point throughput from 1..16 gcc-built caller threads (tools/capi_threads), with the
# combining submit's launch statistics. Optional: HKV_HOST_SETS=1|2.
export HKV_HOST_STATS=1
for t in 1 2 4 8 16; do ./tools/capi_threads throughput $t 1.0 50; done 2>&1
