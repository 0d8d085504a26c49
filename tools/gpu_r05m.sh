#!/bin/bash
# Round 5: the deferred pass's grid (HKV_DEFER_BLOCKS 8 = before, 128 = now) on configs[1] and configs[4],
# kernel traces of configs[4], 3 interleaved runs each.  tools/gpu_r05m.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_workload_gpu.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || exit 11
for k in 8 128; do
  HKV_DEFER_BLOCKS=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$k -o run -- python3 bench.py \
    --config cfg5 --steps 10 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/p$k.log 2>&1 || exit 12
done
for rep in 1 2 3; do
  for k in 8 128; do
    HKV_DEFER_BLOCKS=$k timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/c2_${k}_$rep.log 2>&1 || exit 13
    HKV_DEFER_BLOCKS=$k timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/c5_${k}_$rep.log 2>&1 || exit 14
  done
done
exit 0
