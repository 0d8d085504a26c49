#!/bin/bash
# Round 6: k_local_shared (k_local_fused with each distinct key's lookup shared by the block) -- parity of
# the A/B builds, then the default bench alternating the builds (tools/ab_lib.sh).
#   tools/gpu_r06_lfab.sh TAG lib...   (libs under build_ab/, built with -DHKV_LF_SHARED=NW)
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
k="random_protocol_rounds or max_size_batches or tag_collisions or scripted or local_opcode_mirror or bench_round_mirrored or retry_round_mirrored or membership_change_round or full_size_round"
for lib in "$@"; do
  n=$(basename $(dirname $lib))
  HKV_LIB=$PWD/$lib timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -m gpu -x -q \
    --timeout 240 --timeout-method thread -k "$k" > $out/tests_$n.log 2>&1 || exit 11
done
libs=("")
for lib in "$@"; do libs+=("$PWD/$lib"); done
bash tools/ab_lib.sh $tag "--steps 20 --warmup 5 --policy-steps 0" "${libs[@]}" || exit 12
exit 0
