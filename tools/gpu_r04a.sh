#!/bin/bash
# Round 4, first GPU session: the retry-round tests with the commit audit, the default bench (commit
# breakdown, skew-0 CPU baseline), and per-round dynamics of the retry policies.  tools/gpu_r04a.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_workload_gpu.py -k "retry" > $out/tests.log 2>&1 || exit 12
timeout -k 10 420 python bench.py > $out/bench.log 2>&1 || exit 13
timeout -k 10 300 python tools/round_probe.py --config cfg2 --skew 0 --steps 60 --audit-every 20 > $out/probe_cfg2_skew0.jsonl 2>&1 || exit 4
timeout -k 10 300 python tools/round_probe.py --config cfg2 --skew 3 --steps 30 --audit-every 10 > $out/probe_cfg2_skew3.jsonl 2>&1 || exit 5
timeout -k 10 400 python tools/round_probe.py --config cfg3 --skew 0 --steps 60 > $out/probe_cfg3.jsonl 2>&1 || exit 6
