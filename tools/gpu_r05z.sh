#!/bin/bash
# Round 5: the serving kernel reads the first launch's headers beside its merge scan (HKV_SERVE_SPEC):
# the host-API tests (both ways), then capi_threads at 1 / 8 / 16 threads, interleaved, 3 reps
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_capi_threads.py tests/test_capi.py -m gpu > $out/tests.log 2>&1 || exit 11
HKV_SERVE_SPEC=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_capi_threads.py tests/test_capi.py -m gpu > $out/tests0.log 2>&1 || exit 12
for rep in 1 2 3; do
  for k in 1 0; do
    for t in 1 8 16; do
      HKV_SERVE_SPEC=$k HKV_PART_PROF=1 HKV_HOST_TIMING=1 HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/s${k}_t${t}_$rep.log 2>&1 || exit 13
    done
  done
done
exit 0
