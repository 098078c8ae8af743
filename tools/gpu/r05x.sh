#!/bin/bash
# round 5, call x: the product pass B now on 256-column blocks of 4 waves (8-row stages, 3-deep ring,
# two blocks per CU; 64/128 columns for d <= 64/128): the C = 64 parity tests and the A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_nuts.py -k "64 or 70 or fulldata or fullsize or placement" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passFB_ab_8x2e6.log 2>&1
rc=$?; echo "gemm ab 8x2e6 rc=$rc"; grep -E "parity|median" $O/passFB_ab_8x2e6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passFB_ab_1x25e6.log 2>&1
rc=$?; echo "gemm ab 1x2.5e7 rc=$rc"; grep -E "parity|median" $O/passFB_ab_1x25e6.log
[ $rc -eq 0 ] || exit $rc
[ $rc -eq 0 ] || exit $rc
GEMM_AB_ABL=1 timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_ablations_8x2e6.log 2>&1
rc=$?; echo "gemm ablations rc=$rc"; grep -E "median" $O/passF_ablations_8x2e6.log
exit $rc
