#!/bin/bash
# Per-kernel counters (MI355X_MICROARCH.md, HBM + PMC sections): one rocprofv3 pass per counter
# group, kernel trace only (no runtime/sys traces). FETCH_SIZE and WRITE_SIZE need separate
# passes (TCC slots).
#   tools/pmc.sh TAG "bench args" [group ...]   groups: FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY ..."
tag=$1; bargs=$2; shift 2
groups=("$@"); [ ${#groups[@]} -eq 0 ] && groups=(FETCH_SIZE WRITE_SIZE)
out=$PWD/gpurun_out/$tag/pmc; mkdir -p $out; export TMPDIR=/tmp
i=0
for c in "${groups[@]}"; do
  name=$(echo $c | tr ' ' '+')
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $out/$name -o run -- python3 bench.py $bargs --cpu-seconds 0 --host-api-seconds 0 > $out/$name.log 2>&1 || exit 1
  i=$((i+1))
done
exit 0
