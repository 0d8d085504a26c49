#!/bin/bash
# One bench line and a rocprofv3 kernel trace of the same bench: tools/gpu_prof.sh TAG "bench args"
tag=$1; bargs=$2; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 240 python bench.py $bargs --cpu-seconds 0 --host-api-seconds 0 --retry-steps 0 > $out/bench.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-api-seconds 0 --retry-steps 0 $bargs > $out/prof.log 2>&1 || exit 3
