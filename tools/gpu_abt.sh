#!/bin/bash
# The local-path parity tests, then an A/B of an environment switch (3 alternating reps of a bench),
# then a kernel-stats profile with the switch on.   tools/gpu_abt.sh TAG VAR ["bench args"]
tag=$1; var=$2; bargs=${3:-"--steps 30 --warmup 5"}; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py tests/test_marshal_gpu.py -x -v --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
for rep in 1 2 3; do
  for v in 1 0; do
    env $var=$v timeout -k 10 240 python bench.py $bargs --cpu-seconds 0 --host-api-seconds 0 \
      --policy-steps 0 > $out/b_${v}_$rep.log 2>&1 || exit 12
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py \
  $bargs --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 13
