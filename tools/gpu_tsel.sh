#!/bin/bash
# Selected GPU tests (-k EXPR), then optionally bench lines.   tools/gpu_tsel.sh TAG "expr" ["bench args" ...]
tag=$1; sel=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$sel" > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
[ $rc -ne 0 ] && exit $rc
i=0
for b in "$@"; do
  echo "b$i: $b" >> $out/index.txt
  timeout -k 10 400 python bench.py $b > $out/b$i.log 2>&1 || exit 2
  i=$((i+1))
done
exit 0
