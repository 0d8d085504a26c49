mkdir -p gpurun_out/z3; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_workload_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/z3/wl.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/z3/tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 5 --host-api-seconds 0 > gpurun_out/z3/cfg5.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-api-seconds 0 > gpurun_out/z3/cfg2.log 2>&1 || exit 4
