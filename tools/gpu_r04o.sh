#!/bin/bash
# Round 4: configs[2] (cfg3) steady state and counters. Bench lines after 20 warm-up rounds under fresh
# batches (the plateau) and under retry (the reference's refill_ops, which decays); per-lane value copies
# (HKV_WAVE_COPY=0) against the wave copies; then PMC passes of the fresh plateau: FETCH_SIZE, WRITE_SIZE,
# wave/stall cycles and vector memory instructions, L1->L2 requests.   tools/gpu_r04o.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
b="--config cfg3 --host-api-seconds 0 --policy-steps 0 --cpu-seconds 0"
timeout -k 10 400 python bench.py $b --refill fresh --steps 40 --warmup 20 > $out/bench_fresh.log 2>&1 || exit 11
timeout -k 10 400 python bench.py $b --steps 40 --warmup 20 > $out/bench_retry.log 2>&1 || exit 12
HKV_WAVE_COPY=0 timeout -k 10 300 python bench.py $b --refill fresh --steps 20 --warmup 10 > $out/bench_fresh_lanecopy.log 2>&1 || exit 13
bash tools/pmc.sh $tag "$b --refill fresh --steps 3 --warmup 10" FETCH_SIZE WRITE_SIZE \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum" || exit 14
exit 0
