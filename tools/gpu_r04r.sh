#!/bin/bash
# Round 4: prepass LDS tables and occupancy (library builds in build_ab/, tools/ab_lib.sh), after the
# parity tests of the in-tree build.   tools/gpu_r04r.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
for lib in build_ab/libhermeskv_b512.so build_ab/libhermeskv_b512w7.so build_ab/libhermeskv_b512w8.so; do
  HKV_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread -k "local or small or default" > $out/tests_$(basename $lib .so).log 2>&1 || exit 12
done
bash tools/ab_lib.sh $tag "--steps 30 --warmup 5 --policy-steps 0" "" $PWD/build_ab/libhermeskv_b512.so \
  $PWD/build_ab/libhermeskv_b512w7.so $PWD/build_ab/libhermeskv_b512w8.so || exit 13
exit 0
