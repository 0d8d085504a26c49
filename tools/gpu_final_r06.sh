#!/bin/bash
# Round-6 evidence: the GPU test suite, the default bench line (CPU baselines, policies, host API), a
# rocprofv3 kernel trace + stats of the same bench, its HBM passes (tools/pmc_local.py), configs[2] under
# retry (the reference's policy) and fresh batches with a kernel trace and HBM passes, and configs[4] (cfg5)
# on one GPU.   tools/gpu_final_r06.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gputests.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 12
b="--steps 30 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py $b \
  > $out/prof.log 2>&1 || exit 13
bash tools/pmc.sh $tag "--steps 3 --warmup 2 --policy-steps 0" FETCH_SIZE WRITE_SIZE || exit 14
c3="--config cfg3 --host-api-seconds 0 --policy-steps 0"
timeout -k 10 400 python bench.py $c3 --steps 10 --warmup 50 --cpu-seconds 0 > $out/cfg3_retry.log 2>&1 || exit 15
timeout -k 10 400 python bench.py $c3 --refill fresh --steps 40 --warmup 20 > $out/cfg3_fresh.log 2>&1 || exit 16
mkdir -p $out/cfg3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/cfg3/prof -o run -- python3 bench.py $c3 \
  --refill fresh --steps 10 --warmup 20 --cpu-seconds 0 > $out/cfg3/prof.log 2>&1 || exit 17
bash tools/pmc.sh $tag/cfg3 "$c3 --refill fresh --steps 3 --warmup 20" FETCH_SIZE WRITE_SIZE || exit 18
timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 3 --host-api-seconds 0 --policy-steps 0 > $out/cfg5.log 2>&1 || exit 19
exit 0
