#!/bin/bash
# configs[2] (fresh batches) under environment configurations: a kernel trace each, then 2 interleaved
# bench runs each.  tools/gpu_c3ab.sh TAG CFG...
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
printf '%s\n' "$@" > $out/configs.txt
b="--config cfg3 --refill fresh --steps 10 --warmup 20 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
k=0
for cfg in "$@"; do
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$k -o run -- \
    python3 bench.py $b > $out/p$k.log 2>&1 || exit 14
  k=$((k+1))
done
for rep in 1 2; do
  k=0
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py $b > $out/b_${k}_$rep.log 2>&1 || exit 15
    k=$((k+1))
  done
done
exit 0
