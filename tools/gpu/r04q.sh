#!/bin/bash
# round 4, call q: k_sweep16 with beta in registers AND early release (BREG + PRE) against the
# product (beta image in LDS, early release) and BREG + late release; d = 100 logistic at the
# bench geometry and d = 50 linear; then the C = 16 lpgrad parity tests (d > 108 now runs the
# paired forward with beta in registers).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 240 tools/_bin/sweep16_ab 12500000 8 3 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "parity|median" $O/ab_d100.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 3 10 50 2 > $O/ab_d50.log 2>&1
rc=$?; echo "ab d50 rc=$rc"; grep -E "parity|median" $O/ab_d50.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "lpgrad" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
