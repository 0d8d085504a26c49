#!/bin/bash
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_replica_group_gpu.py -v -s --timeout 100 --timeout-method thread -k "without_host_sync" > $out/synctest.log 2>&1
echo "synctest rc $?" >> $out/synctest.log
