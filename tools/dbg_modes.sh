#!/bin/bash
out=gpurun_out/${TAG:-dbg}; mkdir -p $out; export TMPDIR=/tmp
for m in ${MODES:-0 2 6}; do
  HKV_DBG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out/p$m -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --host-api-seconds 0 --policy-steps 0 > $out/p$m.log 2>&1 || exit 1
done
