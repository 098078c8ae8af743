#!/bin/bash
# round 5, call t: the product pass F now on 128-row tiles (k_gemm_fwd<FAM, 4>): its parity tests, and
# the A/B against 8 waves (256-row tiles) and round 4's kernel at configs[4]'s shape and at bench's
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "64 or 70" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_ab_8x2e6.log 2>&1
rc=$?; echo "gemm ab 8x2e6 rc=$rc"; grep -E "parity|median" $O/passF_ab_8x2e6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passF_ab_1x25e6.log 2>&1
rc=$?; echo "gemm ab 1x2.5e7 rc=$rc"; grep -E "parity|median" $O/passF_ab_1x25e6.log
exit $rc
