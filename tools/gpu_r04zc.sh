#!/bin/bash
# Round 4: sparse refill patches (HKV_SPARSE_PATCH=1: the plan writes refilled slots' patches only, marked
# in the opcode mirror). The parity tests with the defaults and the mirrored rounds with the switch on,
# then 3 alternating bench reps each.   tools/gpu_r04zc.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
HKV_SPARSE_PATCH=1 timeout -k 10 600 python -u -m pytest tests/test_workload_gpu.py tests/test_replica_group_gpu.py -x -v \
  --timeout 120 --timeout-method thread > $out/tests_sparse.log 2>&1 || exit 12
bash tools/gpu_abm.sh $tag "--steps 30 --warmup 5" HKV_SPARSE_PATCH=1 > /dev/null 2>&1 || exit 13
exit 0
