#!/bin/bash
# A/B of bench arguments: tools/ab_args.sh TAG "common args" "variant args" ...  (logs a0.log, a1.log, ...)
tag=$1; common=$2; shift 2
mkdir -p gpurun_out/$tag
i=0
for v in "$@"; do
  timeout -k 10 120 python bench.py $common $v --cpu-seconds 0 --host-api-seconds 0 > gpurun_out/$tag/a$i.log 2>&1 || exit 1
  echo "a$i: $v" >> gpurun_out/$tag/index.txt
  i=$((i+1))
done
