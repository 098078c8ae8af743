#!/bin/bash
# Round 4: residual v4 (k_sweep16) against round 3's k_sweepe at the bench geometry, then the
# sweep parity tests through the library.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
timeout -k 10 120 tools/_bin/sweep16_ab 12500000 8 3 8 100 3 > gpurun_out/r04a/ab_d100_logi.log 2>&1
rc=$?; echo "d100 logistic rc=$rc"; tail -4 gpurun_out/r04a/ab_d100_logi.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/_bin/sweep16_ab 1250000 8 3 20 50 2 > gpurun_out/r04a/ab_d50_lin.log 2>&1
rc=$?; echo "d50 linear rc=$rc"; tail -4 gpurun_out/r04a/ab_d50_lin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04a/pytest_kernels.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -5 gpurun_out/r04a/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/_bin/sweep16_ab 12500000 8 3 8 100 3 > gpurun_out/r04a/ab_d100_logi_2.log 2>&1
rc=$?; echo "d100 logistic (again) rc=$rc"; tail -4 gpurun_out/r04a/ab_d100_logi_2.log
