#!/bin/bash
# Round 5: fused ACKs in the replica group's INV launches: the replica-group and workload GPU tests
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_replica_group_gpu.py tests/test_rccl_gpu.py > $out/tests.log 2>&1 || exit 11
HKV_FUSED_ACKS=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_replica_group_gpu.py -k "loopback" > $out/tests_nofuse.log 2>&1 || exit 12
exit 0
