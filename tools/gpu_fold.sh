#!/bin/bash
# Round 4: slab totals folded into the steady rounds' slabs: the replica-group GPU tests (loopback with the
# oracle mirror, fold on and off; thread-comm steady rounds under sync-debug; gloo-driver; one-rank RCCL).
out=gpurun_out/r04zl; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_rccl_gpu.py tests/test_replica_group_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $out/tests.log 2>&1 || exit 11
exit 0
