#!/bin/bash
# Round 4: parity of the PUT-key mirror and the ACK rows launch, A/Bs of the ACK rows and of k_local_fused's
# elements per lane group, then k_local_pre's timing modes with the PUT-key mirror.  tools/gpu_r04d.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workload_gpu.py tests/test_replica_group_gpu.py tests/test_rccl_gpu.py --maxfail=5 -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 11
HKV_LF_PAIR=4 timeout -k 10 300 python -u -m pytest tests/test_workload_gpu.py -x -q --timeout 200 --timeout-method thread -k "bench_round or retry_round" > $out/tests_lf4.log 2>&1 || exit 11
B="python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for rep in 1 2; do
  for v in 1 0; do HKV_ACK_ROWS=$v HKV_INV_ROWS=$v timeout -k 10 240 $B > $out/ar_${v}_$rep.log 2>&1 || exit 2; done
  for v in 4 2; do HKV_LF_PAIR=$v timeout -k 10 240 $B > $out/lf_${v}_$rep.log 2>&1 || exit 2; done
done
for m in 0 8 16 2 4 1 32; do
  HKV_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$m -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/p$m.log 2>&1 || exit 13
done
