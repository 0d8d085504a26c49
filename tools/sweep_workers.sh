set -e
mkdir -p gpurun_out/sweep
for w in 2048 4096 8192 12288 16384; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --workers $w --cpu-seconds 0 --host-api-seconds 0 > gpurun_out/sweep/w$w.log 2>&1
  echo "w=$w rc=$?"
done
for w in 4096 8192; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --workers $w --cpu-seconds 0 --host-api-seconds 0 --retry > gpurun_out/sweep/r$w.log 2>&1
  echo "retry w=$w rc=$?"
done
