#!/bin/bash
# Round 4: the serving kernel as the default (ring in device memory) with 2 / 4 / 8 launches in flight,
# against launched k_hpart; the full boundary tests first.   tools/gpu_r04za.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_capi_threads.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || exit 11
cfgs=("" "HKV_PART_INFLIGHT=4" "HKV_PART_INFLIGHT=8" "HKV_HOST_SERVE=0")
for rep in 1 2; do
  for k in "${!cfgs[@]}"; do
    for t in 1 8 16; do
      env ${cfgs[$k]} timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/h_${k}_t${t}_$rep.log 2>&1 || exit 12
    done
  done
done
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
exit 0
