#!/bin/bash
# Host-pointer boundary A/B of two library builds (in-tree vs build_ab/head via LD_LIBRARY_PATH): the
# entry-point tests on the in-tree one, then capi_threads at 1 / 8 / 16 threads, interleaved, 3 reps.
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_capi_threads.py tests/test_capi.py -m gpu > $out/tests.log 2>&1 || exit 11
for rep in 1 2 3; do
  for k in 0 1; do
    lp=""; [ $k = 1 ] && lp="$PWD/build_ab/head"
    for t in 1 8 16; do
      LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} HKV_HOST_TIMING=1 HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 \
        > $out/c${k}_t${t}_$rep.log 2>&1 || exit 12
    done
  done
done
exit 0
