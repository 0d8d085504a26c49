#!/bin/bash
# Copy the judged evidence of a tools/gpu_check.sh run into profiles/ (tracked):
#   tools/snapshot.sh TAG NAME  ->  profiles/NAME_bench.json, NAME_kernel_stats.txt, NAME_timeline.txt
tag=$1; name=$2; out=gpurun_out/$tag
grep '^{' $out/bench.log | tail -1 > profiles/${name}_bench.json
f=$(find $out/prof -name "*kernel_stats.csv" | head -1)
{ echo "# rocprofv3 --kernel-trace --stats, same bench command as ${name}_bench.json (gpurun_out/$tag)"; python tools/rocprof_summary.py $f --top 40; } > profiles/${name}_kernel_stats.txt
{ echo "# one bench step from the rocprofv3 kernel trace (tools/step_kernels.py)"; python tools/step_kernels.py $tag; } > profiles/${name}_timeline.txt
if [ -d $out/pmc ]; then
  { echo "# per-kernel PMC means per dispatch (tools/pmc.sh, tools/pmc_summary.py)"; python tools/pmc_summary.py $tag; } > profiles/${name}_pmc.txt
fi
ls -la profiles/${name}_*
