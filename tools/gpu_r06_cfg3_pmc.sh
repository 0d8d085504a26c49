#!/bin/bash
# Round 6, configs[2]: per-kernel HBM counters of the fresh-batch bench with the refill planned as patches
# (default) and in place (--inplace-refill).   tools/gpu_r06_cfg3_pmc.sh TAG
tag=$1; export TMPDIR=/tmp
c3="--config cfg3 --refill fresh --policy-steps 0 --steps 3 --warmup 20"
for mode in fused inplace; do
  extra=""; [ $mode = inplace ] && extra="--inplace-refill"
  bash tools/pmc.sh $tag/$mode "$c3 $extra" FETCH_SIZE WRITE_SIZE "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
    "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES" || exit 11
done
exit 0
