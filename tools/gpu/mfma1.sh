#!/bin/bash
# v4 (fp64 MFMA, 16 chains) first look: parity of the lp/grad hook, then the micro-benchmark.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "lpgrad" > gpurun_out/pytest_v4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_v4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/sweep_micro 12500000 8 100 5 16 > gpurun_out/micro_v4.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro_v4.log
