#!/bin/bash
# Round 4: the host-pointer boundary with callers staging into device memory (HKV_STAGE_VRAM).
# tools/bar_probe first (is fine-grained VRAM host-writable here, and what a call costs each way), then
# the boundary's parity tests with the switch on, then capi_threads throughput A/B (alternating).
#   tools/gpu_r04l.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 60 ./tools/bar_probe 14000 2000 > $out/bar_probe.log 2>&1 || exit 11
grep -q "vram-fg: .*host-writable 1" $out/bar_probe.log || exit 0
HKV_STAGE_VRAM=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_capi_threads.py "tests/test_gpu_parity.py::test_random_rounds_reference_entry_points" > $out/tests_vram.log 2>&1 || exit 12
for rep in 1 2; do
  for v in 0 1; do
    for t in 1 8 16; do
      HKV_STAGE_VRAM=$v timeout -k 10 60 ./tools/capi_threads throughput $t 1.5 50 > $out/h_${v}_t${t}_$rep.log 2>&1 || exit 13
    done
  done
done
HKV_STAGE_VRAM=1 HKV_PART_PROF=64 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput 1 1.5 50 > $out/prof1_vram.log 2>&1 || exit 14
HKV_PART_PROF=64 HKV_HOST_TIMING=1 timeout -k 10 60 ./tools/capi_threads throughput 1 1.5 50 > $out/prof1_pin.log 2>&1 || exit 14
exit 0
