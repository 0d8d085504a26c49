#!/bin/bash
# Same-box A/B of environment switches on the default bench: one rocprofv3 kernel trace per
# configuration, then 3 interleaved bench runs each.  tools/gpu_envab.sh TAG CFG...  ("-" = defaults)
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
printf '%s\n' "$@" > $out/configs.txt
b="--steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
k=0
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=""
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$k -o run -- \
    python3 bench.py $b > $out/p$k.log 2>&1 || exit 14
  k=$((k+1))
done
for rep in 1 2 3; do
  k=0
  for cfg in "$@"; do
    [ "$cfg" = "-" ] && cfg=""
    env $cfg timeout -k 10 200 python bench.py $b > $out/b_${k}_$rep.log 2>&1 || exit 15
    k=$((k+1))
  done
done
exit 0
