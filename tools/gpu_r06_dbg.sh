#!/bin/bash
# Round 6: the host-pointer boundary tests, the local launch under the work-skipping timing modes
# (tools/dbg_modes.sh; HKV_DEBUG_MODES build), then the default bench alternating the in-tree library with the
# builds given (tools/ab_lib.sh).
#   tools/gpu_r06_dbg.sh TAG "modes" lib...
tag=$1; modes=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_capi.py tests/test_capi_threads.py -m gpu -x -q --timeout 240 \
  --timeout-method thread > $out/capi_tests.log 2>&1 || exit 10
TAG=$tag MODES="$modes" bash tools/dbg_modes.sh || exit 11
libs=("")
for lib in "$@"; do libs+=("$PWD/$lib"); done
bash tools/ab_lib.sh $tag "--steps 20 --warmup 5 --policy-steps 0" "${libs[@]}" || exit 12
exit 0
