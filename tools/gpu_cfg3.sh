#!/bin/bash
# configs[2] (cfg3): a bench line and a rocprofv3 kernel trace + stats.   tools/gpu_cfg3.sh TAG ["extra bench args"]
tag=$1; extra=$2; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config cfg3 --steps 10 --warmup 3 --host-api-seconds 0 --policy-steps 0 $extra > $out/bench.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --host-api-seconds 0 --policy-steps 0 --cpu-seconds 0 $extra > $out/prof.log 2>&1 || exit 6
