#!/bin/bash
# The GPU test suite, the default bench line, then configs[2] (cfg3) with its kernel trace.
#   tools/gpu_full.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 2
bash tools/gpu_cfg3.sh $tag/cfg3
