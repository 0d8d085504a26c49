#!/bin/bash
# Round 5: the PUT-key table prepass (HKV_PRE_TABLE) -- parity with it (and with the PUT-key mirror),
# the prepass's workload statistics, kernel stats and a same-box A/B of the four combinations, and
# the work-skipping timing modes of the current prepass (debug build).   tools/gpu_r05b.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
HKV_PRE_TABLE=1 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_workload_gpu.py > $out/t_table.log 2>&1 || exit 11
HKV_PRE_TABLE=1 HKV_PUT_KEYS=1 timeout -k 10 300 $T tests/test_workload_gpu.py > $out/t_table_pk.log 2>&1 || exit 12
timeout -k 10 200 python tools/put_stats.py --steps 12 > $out/put_stats.jsonl 2> $out/put_stats.err || exit 13
cfgs=("" "HKV_PRE_TABLE=1" "HKV_PUT_KEYS=1" "HKV_PRE_TABLE=1 HKV_PUT_KEYS=1")
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
for pk in 0 1; do
  for m in 0 1 2 16 32; do
    HKV_PUT_KEYS=$pk HKV_LIB=$PWD/build_ab/libhermeskv_dbg.so HKV_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $PWD/$out/dbg_${pk}_$m -o run -- python3 tools/round_probe.py --steps 6 > $out/dbg_${pk}_$m.log 2>&1 || true
  done
done
exit 0
