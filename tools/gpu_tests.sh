#!/bin/bash
# GPU parity tests (one process, per-test timeout), then an optional bench line:
#   tools/gpu_tests.sh TAG ["bench args"]
tag=$1; bargs=$2; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
[ -z "$bargs" ] && exit 0
timeout -k 10 300 python bench.py $bargs --host-api-seconds 0 > $out/bench.log 2>&1 || exit 2
