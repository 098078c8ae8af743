#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -X faulthandler -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/kern.log 2>&1
rc=$?; echo "kernel parity rc=$rc"; grep -E "passed|failed|Error" gpurun_out/kern.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/_bin/sweep_micro 12500000 4 100 10 > gpurun_out/micro_v3.log 2>&1
rc=$?; echo "micro v3 rc=$rc"; cat gpurun_out/micro_v3.log
[ $rc -eq 0 ] || exit $rc
STARK_SWEEP=2 timeout -k 10 200 tools/_bin/sweep_micro 12500000 4 100 10 > gpurun_out/micro_v2.log 2>&1
rc=$?; echo "micro v2 rc=$rc"; cat gpurun_out/micro_v2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -X faulthandler -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/all.log 2>&1
rc=$?; echo "all gpu tests rc=$rc"; tail -3 gpurun_out/all.log
