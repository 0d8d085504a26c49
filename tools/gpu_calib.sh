#!/bin/bash
# Counter calibration (tools/calib_bench.hip): the kernels' own timing, then one rocprofv3 --pmc pass
# per counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes, TCC slots),
# and the per-block key sharing of the local launch (tools/put_stats.py).   tools/gpu_calib.sh TAG
tag=$1; out=$PWD/gpurun_out/$tag; mkdir -p $out/pmc; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
timeout -k 10 180 tools/calib_bench > $out/calib.jsonl 2> $out/calib.err || exit 11
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
         "TCC_HIT_sum TCC_MISS_sum" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  name=$(echo $c | tr ' ' '+')
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/pmc/$name -o run -- tools/calib_bench \
    > $out/pmc/$name.log 2>&1 || exit 12
done
timeout -k 10 300 python tools/put_stats.py --steps 8 > $out/put_stats.jsonl 2> $out/put_stats.err || exit 13
exit 0
