#!/bin/bash
# Round 4: parity with the two-stage local launch (prepass beside the VAL batch), then an A/B of it.
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_workload_gpu.py tests/test_gpu_parity.py tests/test_capi_threads.py -v --maxfail=3 --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 11
B="python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for rep in 1 2 3; do
  for v in 1 0; do HKV_PRE_SPLIT=$v timeout -k 10 240 $B > $out/ps_${v}_$rep.log 2>&1 || exit 2; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 13
