#!/bin/bash
# round 2, call a: full -m gpu suite, then the driver's bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest_gpu.log 2>&1
echo "pytest rc=$?"
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
echo "bench rc=$?"
tail -3 gpurun_out/r02a_pytest_gpu.log
