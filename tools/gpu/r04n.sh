#!/bin/bash
# round 4, call n: pass F (64-chain full-data sweep) ablations at d = 1000.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/gemm_ab.log 2>&1
rc=$?; echo "gemm_ab rc=$rc"; grep -E "rows|median" $O/gemm_ab.log
