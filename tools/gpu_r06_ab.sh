#!/bin/bash
# Round 6: parity of the in-tree library on the local-launch tests, then the default bench alternating the
# in-tree library with the builds given (tools/ab_lib.sh), and a kernel trace of the in-tree build.
#   tools/gpu_r06_ab.sh TAG lib...
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
k="random_protocol_rounds or max_size_batches or tag_collisions or scripted or local_opcode_mirror or bench_round_mirrored or retry_round_mirrored or membership_change_round or hades_membership_round or full_size_round or known_answers"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py -m gpu -x -q \
  --timeout 240 --timeout-method thread -k "$k" > $out/tests.log 2>&1 || exit 11
libs=("")
for lib in "$@"; do libs+=("$PWD/$lib"); done
bash tools/ab_lib.sh $tag "--steps 20 --warmup 5 --policy-steps 0" "${libs[@]}" || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py \
  --steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/prof.log 2>&1 || exit 13
exit 0
