#!/bin/bash
# Interleaved A/B of library builds in one GPU session: tools/ab_lib.sh TAG "bench args" lib...
# ("" = the in-tree build). Runs every library twice, alternating, so box drift hits both.
tag=$1; bargs=$2; shift 2
mkdir -p gpurun_out/$tag
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    HKV_LIB=$lib timeout -k 10 120 python bench.py $bargs --cpu-seconds 0 --host-api-seconds 0 > gpurun_out/$tag/l${i}_$rep.log 2>&1 || exit 1
    echo "l$i: ${lib:-in-tree}" >> gpurun_out/$tag/index.txt
    i=$((i+1))
  done
done
