#!/bin/bash
# Round 6: configs[2] under the reference's retry policy (rounds 50-60), refills planned as patches (default)
# against in place (--inplace-refill), alternating.   tools/gpu_r06_cfg3_retry.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
c3="--config cfg3 --host-api-seconds 0 --policy-steps 0 --cpu-seconds 0 --steps 10 --warmup 50"
for rep in 1 2; do
  timeout -k 10 300 python bench.py $c3 > $out/fused_$rep.log 2>&1 || exit 12
  timeout -k 10 300 python bench.py $c3 --inplace-refill > $out/inplace_$rep.log 2>&1 || exit 13
done
exit 0
