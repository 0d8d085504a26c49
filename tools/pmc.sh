#!/bin/bash
# HBM traffic per kernel (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE in
# separate passes (they do not fit one TCC pass), kernel trace only, no runtime/sys traces.
#   tools/pmc.sh TAG "bench args"
tag=$1; bargs=$2
out=$PWD/gpurun_out/$tag/pmc; mkdir -p $out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- python3 bench.py $bargs --cpu-seconds 0 > $out/$c.log 2>&1 || exit 1
done
exit 0
