#!/bin/bash
# Host-pointer boundary: its parity tests, then the throughput diagnostics.   tools/gpu_host.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi_threads.py \
  tests/test_gpu_parity.py -k "reference_entry or capi or threads or shared" > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_hostdiag.sh $tag
