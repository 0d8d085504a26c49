#!/bin/bash
# Round 4: the parity tests, then same-box A/Bs: configs[1] prepass head length (HKV_PRE_HEAD) and
# configs[2] batched big-value wave copies (HKV_VC_BATCH=1: one value at a time), then a configs[2]
# kernel-stats profile with the defaults.   tools/gpu_r04n.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
b2="--steps 30 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
b3="--config cfg3 --refill fresh --steps 20 --warmup 10 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
cfgs=("" "HKV_PRE_HEAD=512" "HKV_PRE_HEAD=256")
for rep in 1 2 3; do
  for k in "${!cfgs[@]}"; do
    env ${cfgs[$k]} timeout -k 10 240 python bench.py $b2 > $out/b_${k}_$rep.log 2>&1 || exit 12
  done
done
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
for rep in 1 2; do
  for v in 0 1; do
    env HKV_VC_BATCH=$([ $v = 1 ] && echo 1 || echo 4) timeout -k 10 300 python bench.py $b3 > $out/c3_${v}_$rep.log 2>&1 || exit 13
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof3 -o run -- python3 bench.py $b3 \
  > $out/prof3.log 2>&1 || exit 14
exit 0
