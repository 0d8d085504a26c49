#!/bin/bash
# configs[2] evidence after a change to its path: the retry policy's number (rounds 50-60), fresh
# batches, a kernel trace + stats of the fresh bench and its HBM passes.   tools/gpu_cfg3_final.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out/cfg3; export TMPDIR=/tmp
c3="--config cfg3 --host-api-seconds 0 --policy-steps 0"
timeout -k 10 400 python bench.py $c3 --steps 10 --warmup 50 --cpu-seconds 0 > $out/cfg3_retry.log 2>&1 || exit 15
timeout -k 10 400 python bench.py $c3 --refill fresh --steps 40 --warmup 20 > $out/cfg3_fresh.log 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/cfg3/prof -o run -- python3 bench.py $c3 \
  --refill fresh --steps 10 --warmup 20 --cpu-seconds 0 > $out/cfg3/prof.log 2>&1 || exit 17
bash tools/pmc.sh $tag/cfg3 "$c3 --refill fresh --steps 3 --warmup 20" FETCH_SIZE WRITE_SIZE || exit 18
exit 0
