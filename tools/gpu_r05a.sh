#!/bin/bash
# Round 5, first session: parity suite, the debug-mode refusal, random-access microbenchmark, the
# prepass's workload statistics, the default bench line.   tools/gpu_r05a.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit 11
HKV_DBG=1 timeout -k 10 60 python bench.py --steps 2 --warmup 1 > $out/dbg_refused.log 2>&1; echo "rc=$?" >> $out/dbg_refused.log
timeout -k 10 120 tools/table_bench > $out/table_bench.json 2> $out/table_bench.err || exit 12
timeout -k 10 200 python tools/put_stats.py --steps 12 > $out/put_stats.jsonl 2> $out/put_stats.err || exit 13
timeout -k 10 400 python bench.py --cpu-seconds 4 > $out/bench.log 2>&1 || exit 14
exit 0
