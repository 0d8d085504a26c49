#!/bin/bash
# fused-refill parity experiments: default, patches written first, local direct off. Stops at any
# exit other than pass (0) / test failure (1).
out=gpurun_out/dbg; mkdir -p $out; export TMPDIR=/tmp
T="tests/test_workload_gpu.py::test_bench_round_mirrored tests/test_workload_gpu.py::test_retry_round_mirrored"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $out/$tag.log 2>&1; rc=$?; echo "$tag rc $rc" >> $out/rc.txt; [ $rc -le 1 ]; }
run a HKV_X=0 && run b HKV_PATCH_APPLY=1 && run c HKV_LOCAL_DIRECT=0
