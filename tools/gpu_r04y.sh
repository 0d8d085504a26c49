#!/bin/bash
# Round 4: big-op INV marshal by whole-wave copies and the virtual peers' timestamp words as plain stores,
# against the previous workload kernels (build_ab/libhermeskv_prevwl.so) and the atomic max
# (HKV_PEER_TS_ATOMIC=1), configs[2] fresh batches, after the parity tests.   tools/gpu_r04y.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py tests/test_marshal_gpu.py -x -v \
  --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 11
b3="--config cfg3 --refill fresh --steps 20 --warmup 10 --policy-steps 0 --cpu-seconds 0 --host-api-seconds 0"
for rep in 1 2; do
  timeout -k 10 300 python bench.py $b3 > $out/d_$rep.log 2>&1 || exit 12
  HKV_LIB=$PWD/build_ab/libhermeskv_prevwl.so timeout -k 10 300 python bench.py $b3 > $out/p_$rep.log 2>&1 || exit 13
  HKV_PEER_TS_ATOMIC=1 timeout -k 10 300 python bench.py $b3 > $out/a_$rep.log 2>&1 || exit 14
done
exit 0
