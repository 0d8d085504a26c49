#!/bin/bash
# Round 4: the replica-group parity tests (retry + skew variants), one-rank RCCL, the gloo bench, and
# configs[2]'s per-round dynamics under retry + skew 3 (the bench's) and fresh batches.  tools/gpu_r04b.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_replica_group_gpu.py tests/test_rccl_gpu.py > $out/tests.log 2>&1 || exit 12
timeout -k 10 300 python tools/round_probe.py --config cfg3 --skew 3 --steps 60 --audit-every 20 > $out/probe_cfg3_skew3.jsonl 2>&1 || exit 13
timeout -k 10 300 python tools/round_probe.py --config cfg3 --skew 3 --refill fresh --steps 40 --audit-every 20 > $out/probe_cfg3_fresh.jsonl 2>&1 || exit 4
