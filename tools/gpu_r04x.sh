#!/bin/bash
# Round 4: k_unique_big keeping its change-detection copies in registers (half the LDS), against the
# previous revision (build_ab/libhermeskv_prevbig.so), configs[2] fresh batches, after the parity tests.
#   tools/gpu_r04x.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
bash tools/ab_lib.sh $tag "--config cfg3 --refill fresh --steps 20 --warmup 10 --policy-steps 0" "" \
  $PWD/build_ab/libhermeskv_prevbig.so || exit 12
exit 0
