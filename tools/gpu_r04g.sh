#!/bin/bash
# Round 4: host-pointer boundary with partitioned launches on several streams: parity tests, then the
# throughput of 1/8/16 gcc-built caller threads with 4 streams against 1.   tools/gpu_r04g.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_capi_threads.py tests/test_capi.py tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -k "capi or reference_entry or known" > $out/tests.log 2>&1 || exit 11
for rep in 1 2; do
  for ns in 4 1; do
    for th in 1 8 16; do
      HKV_PART_STREAMS=$ns timeout -k 10 60 tools/capi_threads throughput $th 1.5 50 >> $out/tp_${ns}.log 2>&1 || exit 12
    done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_workload_gpu.py -x -q --timeout 200 --timeout-method thread > $out/wl.log 2>&1 || exit 13
