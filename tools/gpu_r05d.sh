#!/bin/bash
# Round 5: the reference's shipped semantics (refill_ops retry, skew flags 0) to steady state over 60
# rounds at 64 .. 16384 workers, configs[2] under retry over 60 rounds (its per-round curve), and the
# default bench line (detail.policies.retry now timed over rounds 50-60).   tools/gpu_r05d.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for w in 64 256 1024 4096 16384; do
  timeout -k 10 300 python tools/round_probe.py --config cfg2 --skew 0 --workers $w --steps 60 \
    > $out/skew0_w$w.jsonl 2> $out/skew0_w$w.err || exit 11
done
timeout -k 10 400 python tools/round_probe.py --config cfg3 --skew 3 --refill retry --steps 60 > $out/cfg3_retry.jsonl 2> $out/cfg3_retry.err || exit 12
timeout -k 10 400 python tools/round_probe.py --config cfg3 --skew 0 --refill retry --steps 60 > $out/cfg3_retry_skew0.jsonl 2> $out/cfg3_retry_skew0.err || exit 13
timeout -k 10 400 python bench.py --cpu-seconds 6 > $out/bench.log 2>&1 || exit 14
exit 0
