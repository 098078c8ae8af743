#!/bin/bash
# round 5, call ao: the product pass F on the split stage schedule for d > 112 -- the 64-chain parity
# tests (both families, both schedules), the full-data NUTS tests, and the A/B at both shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ao
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_nuts.py -k "64 or 70 or fulldata or fullsize or placement" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_split_8x2e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-loop|median" $O/passF_split_8x2e6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passF_split_1x25e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-loop|median" $O/passF_split_1x25e6.log
exit $rc
