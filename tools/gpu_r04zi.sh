#!/bin/bash
# Round 4: located entries for the local launch (HKV_LOCAL_HINTS=1: trace keys located once, each slot's word kept by the plan).
# The parity tests with the defaults and the mirrored rounds with the switch on, then 3 alternating bench
# reps each on configs[1] and configs[4].   tools/gpu_r04zh.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py tests/test_capi.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
HKV_LOCAL_HINTS=1 timeout -k 10 600 python -u -m pytest tests/test_workload_gpu.py -x -v \
  --timeout 120 --timeout-method thread > $out/tests_hints.log 2>&1 || exit 12
bash tools/gpu_abm.sh $tag "--steps 30 --warmup 5" HKV_LOCAL_HINTS=1 > /dev/null 2>&1 || exit 13
mkdir -p $out/c5 && for rep in 1 2; do
  for v in 0 1; do
    HKV_LOCAL_HINTS=$v timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --host-api-seconds 0 \
      --policy-steps 0 --cpu-seconds 0 > $out/c5/b_${v}_$rep.log 2>&1 || exit 14
  done
done
exit 0
