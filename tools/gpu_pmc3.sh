#!/bin/bash
# PMC passes of the default bench (FETCH_SIZE, WRITE_SIZE, then TCC hit/miss) for per-kernel HBM
# traffic.   tools/gpu_pmc3.sh TAG ["bench args"]
tag=$1; bargs=${2:-"--steps 3 --warmup 2 --policy-steps 0"}
bash tools/pmc.sh $tag "$bargs" FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" || exit 4
