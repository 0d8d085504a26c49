#!/bin/bash
# Round 4: the host-pointer boundary with device-memory staging under other launch policies: at most
# 1 / 3 launches in flight (HKV_PART_INFLIGHT) and the serving kernel (HKV_HOST_SERVE=1), against the
# defaults, at 1 / 8 / 16 gcc-built threads (2 alternating reps); the boundary's parity tests under the
# serving kernel first.   tools/gpu_r04s.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
HKV_HOST_SERVE=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_capi_threads.py "tests/test_gpu_parity.py::test_random_rounds_reference_entry_points" > $out/tests_serve.log 2>&1 || exit 11
cfgs=("" "HKV_PART_INFLIGHT=1" "HKV_PART_INFLIGHT=3" "HKV_HOST_SERVE=1")
for rep in 1 2; do
  for k in "${!cfgs[@]}"; do
    for t in 1 8 16; do
      env ${cfgs[$k]} timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/h_${k}_t${t}_$rep.log 2>&1 || exit 12
    done
  done
done
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
exit 0
