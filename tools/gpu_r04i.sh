#!/bin/bash
# Round 4: host-pointer boundary, partitioned launches in flight on the table stream (HKV_PART_INFLIGHT).
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
  for inf in 2 4 8 16; do
    for th in 8 16; do
      echo "inflight $inf" >> $out/tp.log
      HKV_PART_INFLIGHT=$inf timeout -k 10 60 tools/capi_threads throughput $th 1.5 50 >> $out/tp.log 2>&1 || exit 12
    done
  done
done
