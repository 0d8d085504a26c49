#!/bin/bash
# Round-3 profile set: the default bench line (CPU baseline, policies, host API), a rocprofv3 kernel
# trace + stats of the same bench, the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the local launch,
# and a configs[2] (cfg3) bench line with its kernel trace.   tools/gpu_final3.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 10 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 3
bash tools/pmc.sh $tag "--steps 3 --warmup 2 --policy-steps 0" FETCH_SIZE WRITE_SIZE || exit 4
timeout -k 10 400 python bench.py --config cfg3 --steps 10 --warmup 3 --host-api-seconds 0 --policy-steps 0 > $out/cfg3.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof_cfg3 -o run -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --host-api-seconds 0 --policy-steps 0 > $out/prof_cfg3.log 2>&1 || exit 6
