#!/bin/bash
# Round profile set: the default bench line, a rocprofv3 kernel trace + stats of the same bench,
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE) the local launch's traffic comes from.
#   tools/gpu_final.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --retry-steps 0 > $out/prof.log 2>&1 || exit 3
bash tools/pmc.sh $tag "--steps 3 --warmup 1 --retry-steps 0" FETCH_SIZE WRITE_SIZE || exit 4
