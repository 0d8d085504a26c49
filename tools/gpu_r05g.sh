#!/bin/bash
# Round 5: the fused pass with more loads in flight per wave -- two chunks per wave (HKV_LF_2C) and the
# software-pipelined persistent pass (HKV_LF_PIPE, 16 / 32 waves per CU): parity, then a same-box A/B.
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
HKV_LF_2C=1 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_workload_gpu.py > $out/t_2c.log 2>&1 || exit 11
HKV_LF_PIPE=1 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_workload_gpu.py > $out/t_pipe.log 2>&1 || exit 12
cfgs=("" "HKV_LF_2C=1" "HKV_LF_PIPE=1" "HKV_LF_PIPE=1 HKV_LF_PIPE_WAVES=16")
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
b="--steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for k in "${!cfgs[@]}"; do
  env ${cfgs[$k]} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$k -o run -- \
    python3 bench.py $b > $out/p$k.log 2>&1 || exit 14
done
for rep in 1 2 3; do
  for k in "${!cfgs[@]}"; do
    env ${cfgs[$k]} timeout -k 10 200 python bench.py $b > $out/b_${k}_$rep.log 2>&1 || exit 15
  done
done
exit 0
