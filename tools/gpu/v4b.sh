#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lpgrad" > gpurun_out/pytest_v4b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_v4b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/sweep_micro 12500000 8 100 5 16 > gpurun_out/micro_v4d.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -E "v4|sweep|stream" gpurun_out/micro_v4d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/sweep_micro 4000000 4 1000 3 64 > gpurun_out/micro_v5b.log 2>&1
rc=$?; echo "micro5 rc=$rc"; cat gpurun_out/micro_v5b.log
