#!/bin/bash
# Round 5: bucket-side F diagnosis: line_bench (footprint), then new lib with HKV_BSIDE=1/0 against head
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 tools/line_bench > $out/line_bench.json || exit 10
b="--steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
cfgs=("HKV_BSIDE=1" "HKV_BSIDE=0" "HKV_LIB=build_ab/libhermeskv_head.so")
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
for k in "${!cfgs[@]}"; do
  env ${cfgs[$k]} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$k -o run -- \
    python3 bench.py $b > $out/p$k.log 2>&1 || exit 14
done
exit 0
