#!/bin/bash
# Round 5: k_scan_cap's held total reduced in parallel: replica-group GPU tests, then the 8-replica probe traced
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_replica_group_gpu.py tests/test_marshal_gpu.py > $out/tests.log 2>&1 || exit 11
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 tools/group_phase_probe.py 8 20000000 4096 10 > $out/probe.json 2> $out/probe.err || exit 12
timeout -k 10 400 python3 tools/group_phase_probe.py 8 20000000 4096 10 > $out/probe2.json 2> $out/probe2.err || exit 13
