#!/bin/bash
# configs[4] on one GPU under a rocprofv3 kernel trace.  tools/gpu_cfg5prof.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py \
  --config cfg5 --steps 10 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 11
