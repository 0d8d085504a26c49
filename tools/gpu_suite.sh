#!/bin/bash
# The whole GPU test suite and one default bench line.  tools/gpu_suite.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/gputests.log 2>&1 || exit 11
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 12
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 13
exit 0
