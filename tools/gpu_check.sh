#!/bin/bash
# One GPU call: parity tests, then (only if they pass) bench runs, optionally a rocprofv3 stats run.
#   tools/gpu_check.sh TAG "bench args" [profile]
tag=$1; bargs=$2; prof=$3
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $out/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py $bargs > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc" >> $out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$prof" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python bench.py $bargs --cpu-seconds 0 > $out/prof.log 2>&1
  echo "prof rc=$?" >> $out/prof.log
fi
exit 0
