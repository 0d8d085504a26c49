#!/bin/bash
# Round 5: packed slabs on the live-peer prefix after a failure: the workload GPU tests, then configs[4]
# with and without it (3 interleaved runs each).  tools/gpu_r05l.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_workload_gpu.py > $out/tests.log 2>&1 || exit 11
b="--config cfg5 --steps 20 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for rep in 1 2 3; do
  for k in 0 1; do
    HKV_PACKED_PREFIX=$k timeout -k 10 300 python bench.py $b > $out/b_${k}_$rep.log 2>&1 || exit 12
  done
done
exit 0
