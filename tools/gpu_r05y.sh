#!/bin/bash
# Round 5: keys in flight per lane group in the prepass (HKV_PRE_PAIR builds in build_ab/)
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
cfgs=(HKV_X=0)
for lib in build_ab/libhermeskv_pp*.so; do
  HKV_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "local or default" > $out/tests_$(basename $lib .so).log 2>&1 || exit 11
  cfgs+=(HKV_LIB=$lib)
done
bash tools/gpu_envab.sh $tag/ab "${cfgs[@]}" || exit 12
