#!/bin/bash
# A/B of an environment switch, 3 alternating reps of a 30-step bench each:
#   tools/gpu_ab3.sh TAG VAR "bench args"
tag=$1; var=$2; bargs=$3
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in 1 0; do
    env $var=$v timeout -k 10 240 python bench.py --steps 30 --warmup 5 $bargs --cpu-seconds 0 --host-api-seconds 0 \
      --retry-steps 0 > $out/b_${v}_$rep.log 2>&1 || exit 2
  done
done
