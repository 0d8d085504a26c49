#!/bin/bash
# Round 6, configs[2]: the tests of the big-op paths, then the fresh-batch bench alternating the in-tree library
# with the refill planned as patches (default), the same in place (--inplace-refill) and each library given
# (HKV_LIB, planned), then a kernel trace + stats of the in-tree default.   tools/gpu_r06_cfg3.sh TAG [lib...]
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_workload_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "big_patches or bench_round_mirrored or rmw_semantics or refill_plan or big_op" > $out/tests.log 2>&1 || exit 11
c3="--config cfg3 --refill fresh --host-api-seconds 0 --policy-steps 0 --cpu-seconds 0 --steps 20 --warmup 20"
for rep in 1 2; do
  timeout -k 10 200 python bench.py $c3 > $out/fused_$rep.log 2>&1 || exit 12
  timeout -k 10 200 python bench.py $c3 --inplace-refill > $out/inplace_$rep.log 2>&1 || exit 13
  i=0
  for lib in "$@"; do
    HKV_LIB=$PWD/$lib timeout -k 10 200 python bench.py $c3 > $out/lib${i}_$rep.log 2>&1 || exit 14
    i=$((i+1))
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/prof -o run -- python3 bench.py \
  --config cfg3 --refill fresh --host-api-seconds 0 --policy-steps 0 --cpu-seconds 0 --steps 10 --warmup 20 \
  > $out/prof.log 2>&1 || exit 15
exit 0
