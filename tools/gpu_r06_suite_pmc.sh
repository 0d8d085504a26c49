#!/bin/bash
# Round 6: the GPU test suite, one default bench line, a kernel trace + stats of the bench, and PMC passes
# for the local launch's instruction mix, issue stalls and DRAM-vs-Infinity-Cache reads.
#   tools/gpu_r06_suite_pmc.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/gputests.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || exit 12
b="--steps 30 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py $b \
  > $out/prof.log 2>&1 || exit 13
bash tools/pmc.sh $tag "--steps 3 --warmup 2 --policy-steps 0" FETCH_SIZE WRITE_SIZE \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" \
  "SQ_WAIT_ANY SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" || exit 14
exit 0
