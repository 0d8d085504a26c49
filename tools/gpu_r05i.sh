#!/bin/bash
# Round 5: F words beside the buckets (128-B index stride): the GPU suite, then an interleaved A/B
# against the previous library (build_ab/libhermeskv_head.so) with kernel traces.  tools/gpu_r05i.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit 11
libs=("" "build_ab/libhermeskv_head.so")
b="--steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for k in "${!libs[@]}"; do
  HKV_LIB=${libs[$k]} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$k -o run -- \
    python3 bench.py $b > $out/p$k.log 2>&1 || exit 14
done
for rep in 1 2 3; do
  for k in "${!libs[@]}"; do
    HKV_LIB=${libs[$k]} timeout -k 10 200 python bench.py $b > $out/b_${k}_$rep.log 2>&1 || exit 15
  done
done
exit 0
