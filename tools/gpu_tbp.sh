#!/bin/bash
# GPU tests, then (unless they timed out or crashed) one bench line and a rocprofv3 kernel trace
# of a short bench.   tools/gpu_tbp.sh TAG "pytest args" "bench args"
tag=$1; targs=$2; bargs=$3
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread $targs > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $out/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py $bargs > $out/bench.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py --steps 10 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 3
