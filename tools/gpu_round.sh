#!/bin/bash
# One GPU call: parity tests (one process, per-test timeout), then a bench line, then a short
# rocprofv3 kernel trace of the same bench.
#   tools/gpu_round.sh TAG "bench args" [notest]
tag=$1; bargs=$2; skip=$3
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
if [ "$skip" != "notest" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1; rc=$?
  echo "tests rc=$rc" >> $out/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python bench.py $bargs > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc" >> $out/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --host-api-seconds 0 --retry-steps 0 $bargs > $out/prof.log 2>&1
echo "prof rc=$?" >> $out/prof.log
exit 0
