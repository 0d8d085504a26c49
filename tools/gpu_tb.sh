#!/bin/bash
# GPU tests then (unless they timed out or crashed) one bench line.
#   tools/gpu_tb.sh TAG "pytest args" "bench args"
tag=$1; targs=$2; bargs=$3
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread $targs > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py $bargs > $out/bench.log 2>&1
