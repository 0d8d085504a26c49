#!/bin/bash
# Round 6: the local launch under the work-skipping timing modes (tools/dbg_modes.sh; HKV_DEBUG_MODES build),
# then the default bench alternating the in-tree library with the builds given (tools/ab_lib.sh).
#   tools/gpu_r06_dbg.sh TAG "modes" lib...
tag=$1; modes=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
TAG=$tag MODES="$modes" bash tools/dbg_modes.sh || exit 11
libs=("")
for lib in "$@"; do libs+=("$PWD/$lib"); done
bash tools/ab_lib.sh $tag "--steps 20 --warmup 5 --policy-steps 0" "${libs[@]}" || exit 12
exit 0
