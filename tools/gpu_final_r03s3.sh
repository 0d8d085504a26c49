#!/bin/bash
# Round-3 session-3 evidence: the default bench line (CPU baseline, policies, host API), a rocprofv3 kernel
# trace + stats of the same bench, the PMC passes, configs[2] (cfg3, 20 steps, + kernel trace) and
# configs[4] (cfg5) on one GPU.   tools/gpu_final_r03s3.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 10 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 3
bash tools/pmc.sh $tag "--steps 3 --warmup 2 --policy-steps 0" FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" || exit 4
timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --host-api-seconds 0 --policy-steps 0 > $out/cfg3.log 2>&1 || exit 5
mkdir -p $out/cfg3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/cfg3/prof -o run -- python3 bench.py --config cfg3 --steps 10 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/cfg3/prof.log 2>&1 || exit 6
timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 3 --host-api-seconds 0 --policy-steps 0 > $out/cfg5.log 2>&1 || exit 7
