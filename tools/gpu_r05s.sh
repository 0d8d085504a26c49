#!/bin/bash
# Round 5: the fused INV marshal + ACK offsets + peer ACKs: its unit test, the workload and parity GPU
# tests, then an interleaved A/B on the default bench (HKV_FUSED_MARSHAL=1 / 0) with kernel traces
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_marshal_gpu.py tests/test_workload_gpu.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || exit 11
bash tools/gpu_envab.sh $tag/ab HKV_FUSED_MARSHAL=1 HKV_FUSED_MARSHAL=0 || exit 12
