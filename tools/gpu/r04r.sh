#!/bin/bash
# round 4, call r: k_sweep16 with beta always in registers (early release up to d = 108
# logistic, every d linear) against the committed kernel (beta image in LDS); d = 100 logistic
# at the bench geometry and d = 50 linear; then every GPU kernel test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 240 tools/_bin/sweep16_ab 12500000 8 5 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "parity|median" $O/ab_d100.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 3 10 50 2 > $O/ab_d50.log 2>&1
rc=$?; echo "ab d50 rc=$rc"; grep -E "parity|median" $O/ab_d50.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
