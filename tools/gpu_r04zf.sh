#!/bin/bash
# Round 4: the driver's round-end sequence, twice: the GPU test suite, smoke() and the default bench.
#   tools/gpu_r04zf.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests_$rep.log 2>&1 || exit 11
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$rep.log 2>&1 || exit 12
  timeout -k 10 400 python bench.py > $out/bench_$rep.log 2>&1 || exit 13
done
exit 0
