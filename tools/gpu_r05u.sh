#!/bin/bash
# Round 5: the prepass's block size (HKV_PRE_ELEMS builds in build_ab/): parity tests per build, then the A/B
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for lib in build_ab/libhermeskv_pre2048.so build_ab/libhermeskv_pre4096.so; do
  HKV_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_workload_gpu.py > $out/tests_$(basename $lib .so).log 2>&1 || exit 11
done
bash tools/gpu_envab.sh $tag/ab HKV_X=0 HKV_LIB=build_ab/libhermeskv_pre2048.so HKV_LIB=build_ab/libhermeskv_pre4096.so || exit 12
