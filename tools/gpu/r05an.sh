#!/bin/bash
# round 5, call an (y read after the last part): pass F with a split stage schedule (the first 8 stages of a tile carry one
# epilogue part each, a constant; the rest none) against the product loop (one part dispatch per stage)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05an
mkdir -p $O
GEMM_AB_ABL=1 timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_split_8x2e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-split|median F" $O/passF_split_8x2e6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 3 > $O/passF_split_1x25e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-split|median F" $O/passF_split_1x25e6.log
exit $rc
