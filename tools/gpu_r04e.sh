#!/bin/bash
# Round 4: the thread-comm sync test alone (debugging a hang), then the rest of r04d.  tools/gpu_r04e.sh TAG
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_replica_group_gpu.py -v --timeout 100 --timeout-method thread -k "without_host_sync" > $out/synctest.log 2>&1
echo "synctest rc $?" >> $out/synctest.log
timeout -k 10 200 python -u -m pytest tests/test_rccl_gpu.py -v --timeout 150 --timeout-method thread > $out/rccl.log 2>&1 || exit 11
B="python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0"
for rep in 1 2; do
  for v in 1 0; do HKV_ACK_ROWS=$v HKV_INV_ROWS=$v timeout -k 10 240 $B > $out/ar_${v}_$rep.log 2>&1 || exit 2; done
  for v in 4 2; do HKV_LF_PAIR=$v timeout -k 10 240 $B > $out/lf_${v}_$rep.log 2>&1 || exit 2; done
done
for m in 0 8 16 2 4 1 32; do
  HKV_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$m -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/p$m.log 2>&1 || exit 13
done
