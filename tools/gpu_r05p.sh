#!/bin/bash
# Round 5: kernel trace of the 8-replica group on one GPU (tools/group_phase_probe.py)
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 tools/group_phase_probe.py 8 20000000 4096 10 > $out/probe.json 2> $out/probe.err || exit 11
