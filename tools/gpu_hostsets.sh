#!/bin/bash
# Host-pointer boundary: parity tests, then throughput against the partitioned launches in flight.
#   tools/gpu_hostsets.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi_threads.py \
  tests/test_gpu_parity.py -k "reference_entry or capi or threads or shared" > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
[ $rc -ne 0 ] && exit $rc
for s in 1 2 4 8; do
  for t in 1 8 16; do
    echo "inflight $s threads $t: $(HKV_PART_INFLIGHT=$s HKV_HOST_STATS=1 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput $t 2 50 2>&1 | tr '\n' ' ')" >> $out/sets.log || exit 5
  done
done
HKV_HOST_SERVE=0 HKV_PART_PROF=64 timeout -k 10 60 ./tools/capi_threads throughput 8 2 50 > $out/prof8.log 2>&1 || exit 6
for t in 1 8 16; do echo "serve=0 threads $t: $(HKV_HOST_SERVE=0 HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 2 50 2>&1 | tr "\n" " ")" >> $out/sets.log || exit 7; done
