#!/bin/bash
# Paired serving kernel: the host-API parity tests with it on, then tools/gpu_hpab.sh's A/B.  TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out
HKV_SERVE_PAIR=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_capi_threads.py tests/test_capi.py -m gpu > $out/tests_pair.log 2>&1 || exit 10
bash tools/gpu_hpab.sh $tag HKV_SERVE_PAIR=0 HKV_SERVE_PAIR=1
