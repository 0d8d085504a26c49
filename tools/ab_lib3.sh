#!/bin/bash
# Interleaved A/B of library builds, 3 reps of a 30-step bench each: tools/ab_lib3.sh TAG "bench args" lib...
# ("" = the in-tree build)
tag=$1; bargs=$2; shift 2
mkdir -p gpurun_out/$tag
for rep in 1 2 3; do
  i=0
  for lib in "$@"; do
    HKV_LIB=$lib timeout -k 10 240 python bench.py --steps 30 --warmup 5 $bargs --cpu-seconds 0 --host-api-seconds 0 \
      --retry-steps 0 > gpurun_out/$tag/l${i}_$rep.log 2>&1 || exit 1
    i=$((i+1))
  done
done
