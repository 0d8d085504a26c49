#!/bin/bash
# A/B of an environment switch in one GPU session, optionally after the GPU parity tests:
#   tools/gpu_ab_env.sh TAG VAR "bench args" [tests]
# runs bench.py twice with VAR=1 and twice with VAR=0, alternating, so box drift hits both.
tag=$1; var=$2; bargs=$3; tests=$4
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || exit 1
fi
for rep in 1 2 3; do
  for v in 1 0; do
    env $var=$v timeout -k 10 240 python bench.py $bargs --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 \
      > $out/b_${v}_$rep.log 2>&1 || exit 2
  done
done
