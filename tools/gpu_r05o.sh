#!/bin/bash
# Round 5: the 8-replica group on one GPU (tools/group_phase_probe.py), fused ACKs on / off, twice each
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
  for f in 1 0; do
    HKV_FUSED_ACKS=$f timeout -k 10 400 python tools/group_phase_probe.py 8 20000000 4096 10 > $out/g${f}_$rep.json 2> $out/g${f}_$rep.err || exit 11
  done
done
exit 0
