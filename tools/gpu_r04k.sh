#!/bin/bash
# Round 4: configs[2] (cfg3) steady state. Bench lines after 20 warm-up rounds under fresh batches (the
# plateau) and under retry (the reference's refill_ops, which decays), a kernel-stats profile and the
# FETCH_SIZE / WRITE_SIZE PMC passes of the fresh plateau.   tools/gpu_r04k.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
b="--config cfg3 --host-api-seconds 0 --policy-steps 0"
timeout -k 10 400 python bench.py $b --refill fresh --steps 40 --warmup 20 --cpu-seconds 0 > $out/bench_fresh.log 2>&1 || exit 11
timeout -k 10 400 python bench.py $b --steps 40 --warmup 20 --cpu-seconds 0 > $out/bench_retry.log 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py $b \
  --refill fresh --steps 10 --warmup 20 --cpu-seconds 0 > $out/prof.log 2>&1 || exit 13
bash tools/pmc.sh $tag "$b --refill fresh --steps 5 --warmup 20" FETCH_SIZE WRITE_SIZE || exit 14
