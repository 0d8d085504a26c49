#!/bin/bash
# Round-3 GPU call: the GPU test suite (one process, per-test timeout), then bench lines for the
# given variants.  tools/gpu_r03.sh TAG "common bench args" ["variant args" ...]   (TESTS=0 skips tests)
tag=$1; common=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${TESTSEL} > $out/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $out/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for v in "$@"; do
  echo "b$i: $common $v" >> $out/index.txt
  timeout -k 10 300 python bench.py $common $v > $out/b$i.log 2>&1 || exit 2
  i=$((i+1))
done
exit 0
