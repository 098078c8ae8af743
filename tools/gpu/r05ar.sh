#!/bin/bash
# round 5, call ar: pass B with X's LDS-DMA non-temporal against the product, 5 rounds at both shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ar
mkdir -p $O
GEMM_AB_NT=1 timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passB_ntX_8x2e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity B-ntX|median B" $O/passB_ntX_8x2e6.log; [ $rc -eq 0 ] || exit $rc
GEMM_AB_NT=1 timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passB_ntX_1x25e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity B-ntX|median B" $O/passB_ntX_1x25e6.log
exit $rc
