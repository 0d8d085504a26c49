#!/bin/bash
# Round 4: the serving kernel with its ring and stop word in device memory (polled in HBM), against the
# defaults; the boundary's parity tests under the serving kernel first.   tools/gpu_r04z.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
HKV_HOST_SERVE=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_capi_threads.py "tests/test_gpu_parity.py::test_random_rounds_reference_entry_points" > $out/tests_serve.log 2>&1 || exit 11
cfgs=("" "HKV_HOST_SERVE=1")
for rep in 1 2 3; do
  for k in "${!cfgs[@]}"; do
    for t in 1 8 16; do
      env ${cfgs[$k]} timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/h_${k}_t${t}_$rep.log 2>&1 || exit 12
    done
  done
done
HKV_HOST_SERVE=1 HKV_PART_PROF=64 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput 1 1.5 50 > $out/prof1_serve.log 2>&1 || exit 13
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
exit 0
