#!/bin/bash
# Host-pointer boundary A/B: the host-API parity tests, then capi_threads throughput at 1 / 8 / 16
# threads for each configuration, interleaved twice, with k_hserve's phases.  tools/gpu_hpab.sh TAG CFG...
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_capi_threads.py tests/test_capi.py -m gpu > $out/tests.log 2>&1 || exit 11
printf '%s\n' "$@" > $out/configs.txt
for rep in 1 2; do
  k=0
  for cfg in "$@"; do
    for t in 1 8 16; do
      env $cfg HKV_PART_PROF=1 HKV_HOST_TIMING=1 HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 \
        > $out/c${k}_t${t}_$rep.log 2>&1 || exit 12
    done
    k=$((k+1))
  done
done
exit 0
