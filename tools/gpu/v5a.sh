#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lpgrad" > gpurun_out/pytest_v5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_v5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/sweep_micro 4000000 4 1000 3 64 > gpurun_out/micro_v5.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro_v5.log
