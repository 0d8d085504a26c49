#!/bin/bash
# Round 4: the host boundary after the exit hook (serving kernel default): its tests, and the
# throughput tool at 1 / 8 threads.   tools/gpu_r04ze.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_capi_threads.py \
  "tests/test_gpu_parity.py::test_random_rounds_reference_entry_points" > $out/tests.log 2>&1 || exit 11
for t in 1 8; do
  timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/h_t$t.log 2>&1 || exit 12
done
exit 0
