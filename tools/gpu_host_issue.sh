#!/bin/bash
# host-side cost of the bench round: host_issue.py (wall / wait / busy per step) and a cProfile of it
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python tools/host_issue.py --steps 60 > $out/host_issue.json 2> $out/host_issue.err || exit 11
timeout -k 10 300 python -m cProfile -o $out/host_issue.pstats tools/host_issue.py --steps 200 > $out/host_issue2.json 2>&1 || exit 12
python -c "import pstats; pstats.Stats('$out/host_issue.pstats').sort_stats('tottime').print_stats(40)" > $out/pstats.txt || exit 13
