#!/bin/bash
# round 4, call o: pass F variants (128-row tiles, 16-column stages) against the product pass F,
# parity of each after pass B + the reduction; a ragged row count for the tails.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/gemm_ab.log 2>&1
rc=$?; echo "gemm_ab rc=$rc"; grep -E "parity|rows|median" $O/gemm_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/_bin/gemm_ab 1999937 8 1 > $O/gemm_ab_ragged.log 2>&1
rc=$?; echo "gemm_ab ragged rc=$rc"; grep -E "parity|median" $O/gemm_ab_ragged.log
