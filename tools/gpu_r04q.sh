#!/bin/bash
# Round 4: big ops refilled in place one wave per worker (HKV_REFILL_ST_W) and big commits by wave
# block copies. The parity tests (big objects, RMWs and the configs[2] round mirrored), then configs[2]
# fresh-batch A/B (2 alternating reps) and a kernel-stats profile with the defaults.   tools/gpu_r04q.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
b3="--config cfg3 --refill fresh --steps 20 --warmup 10 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for rep in 1 2; do
  for v in 1 0; do
    HKV_REFILL_ST_W=$v timeout -k 10 300 python bench.py $b3 > $out/c3_${v}_$rep.log 2>&1 || exit 12
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof3 -o run -- python3 bench.py $b3 \
  > $out/prof3.log 2>&1 || exit 13
exit 0
