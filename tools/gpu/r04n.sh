#!/bin/bash
# round 4, call n: pass F (64-chain full-data sweep) ablations at d = 1000.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/gemm_ab.log 2>&1
rc=$?; echo "gemm_ab rc=$rc"; grep -E "rows|median" $O/gemm_ab.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_nuts.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
