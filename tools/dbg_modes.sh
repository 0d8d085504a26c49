#!/bin/bash
# The local launch timed under the work-skipping modes (HKV_DBG bits; k_local_pre: 1 no offers, 2 no lookups,
# 4 no head filter, 8 empty kernel, 16 loads only; k_local_fused: 64 no resolve, 128 no lookups, 256 no op
# write-back, 512 no F loads, 1024 no per-element scratch and state-mirror stores). Results are invalid by
# design, so the modes exist
# only in a separate build (-DHKV_DEBUG_MODES) and run through tools/round_probe.py: bench.py refuses
# both HKV_DBG and such a library.
#   here:        tools/dbg_modes.sh build      (build_ab/libhermeskv_dbg.so)
#   on the box:  TAG=dbg MODES="0 2 16" tools/dbg_modes.sh
if [ "$1" = build ]; then
  mkdir -p build_ab && cd hermes_amd/csrc && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics \
    -DHKV_DEBUG_MODES -shared -o ../../build_ab/libhermeskv_dbg.so hkv_batch.hip hkv_kernels.hip hkv_runtime.hip \
    hkv_workload.hip hkv_hades.cpp
  exit $?
fi
out=gpurun_out/${TAG:-dbg}; mkdir -p $out; export TMPDIR=/tmp
for m in ${MODES:-0 2 6}; do
  HKV_LIB=$PWD/build_ab/libhermeskv_dbg.so HKV_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $PWD/$out/p$m -o run -- python3 tools/round_probe.py --steps 6 > $out/p$m.log 2>&1 || exit 1
done
