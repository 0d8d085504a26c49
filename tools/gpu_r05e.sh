#!/bin/bash
# Round 5: prepass without tags (HKV_PRE_NOTAG) parity + A/B against speculative F loads alone, then
# tools/gpu_r05d.sh's steady-state probes.   tools/gpu_r05e.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
HKV_PRE_NOTAG=1 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_workload_gpu.py > $out/t_notag.log 2>&1 || exit 11
cfgs=("" "HKV_LF_FSPEC=1" "HKV_PRE_NOTAG=1")
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
bash tools/gpu_r05d.sh $tag/probes || exit 16
exit 0
