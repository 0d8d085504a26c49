#!/bin/bash
# Host-pointer boundary A/B: the entry-point tests once, then tools/capi_threads throughput at 1 / 8 / 16
# threads, alternating reps, for the defaults and each environment switch given.
#   tools/gpu_hostab.sh TAG VAR=VAL ...            (outputs h_<k>_t<threads>_<rep>.log, k = 0: defaults)
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_capi_threads.py tests/test_capi.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
cfgs=("" "$@")
for rep in 1 2; do
  for k in "${!cfgs[@]}"; do
    for t in 1 8 16; do
      env ${cfgs[$k]} HKV_HOST_STATS=1 timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/h_${k}_t${t}_$rep.log 2>&1 || exit 12
    done
  done
done
printf '%s\n' "${cfgs[@]}" > $out/configs.txt
exit 0
