#!/bin/bash
# Round 4: located entries as a compile-time kernel variant (the default kernels carry no hint branch:
# k_local_fused<2> 47 VGPRs again, 56 with the branch). Parity tests with the defaults and with both hint
# switches on, then 3 alternating bench reps: defaults against HKV_PHYS_HINTS=1 HKV_LOCAL_HINTS=1.
#   tools/gpu_r04zj.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py tests/test_capi.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
HKV_LOCAL_HINTS=1 HKV_PHYS_HINTS=1 timeout -k 10 600 python -u -m pytest tests/test_workload_gpu.py -x -v \
  --timeout 120 --timeout-method thread > $out/tests_hints.log 2>&1 || exit 12
bash tools/gpu_abm.sh $tag "--steps 30 --warmup 5" "HKV_PHYS_HINTS=1 HKV_LOCAL_HINTS=1" > /dev/null 2>&1 || exit 13
exit 0
