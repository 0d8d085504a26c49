#!/bin/bash
# Several environment switches against the defaults on one box: the parity tests once, then 3
# alternating reps of the bench for the defaults and for each switch.
#   tools/gpu_abm.sh TAG "bench args" VAR=VAL [VAR=VAL ...]      (outputs b_<k>_<rep>.log, k = 0: defaults)
tag=$1; bargs=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py tests/test_marshal_gpu.py -x -v \
  --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 11
cfgs=("" "$@")
for rep in 1 2 3; do
  for k in "${!cfgs[@]}"; do
    env ${cfgs[$k]} timeout -k 10 240 python bench.py $bargs --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 \
      > $out/b_${k}_$rep.log 2>&1 || exit 12
  done
done
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
exit 0
