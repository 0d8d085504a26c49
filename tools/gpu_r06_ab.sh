#!/bin/bash
# Round 6: the GPU test suite on the in-tree library, then the default bench alternating the in-tree library
# with the builds given (tools/ab_lib.sh), and a kernel trace of the in-tree build.
#   tools/gpu_r06_ab.sh TAG lib...
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || exit 11
libs=("")
for lib in "$@"; do libs+=("$PWD/$lib"); done
bash tools/ab_lib.sh $tag "--steps 20 --warmup 5 --policy-steps 0" "${libs[@]}" || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py \
  --steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 13
exit 0
