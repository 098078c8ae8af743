#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 tools/_bin/sweep_micro 12500000 4 100 10 > gpurun_out/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts.py -m gpu -q -k adaptive --timeout 120 --timeout-method thread > gpurun_out/jit_tests.log 2>&1
rc=$?; echo "jit tests rc=$rc"; tail -3 gpurun_out/jit_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/chain_diag.py --rows 2.5e7 --adapt 300 --samples 60 --jitter 0.5 > gpurun_out/diag_jit.log 2>&1
echo "diag jit rc=$?"; grep -E "iters" gpurun_out/diag_jit.log | tail -2
