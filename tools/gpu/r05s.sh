#!/bin/bash
# round 5, call s: pass F with 128-row tiles (4 waves, two blocks per CU) and 256-row tiles (8 waves, one
# block per CU) against the product, at configs[4]'s shape (8 x 2e6 rows) and at bench's (1 x 2.5e7 rows)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_w_ab_8x2e6.log 2>&1
rc=$?; echo "gemm ab 8x2e6 rc=$rc"; grep -E "parity|median" $O/passF_w_ab_8x2e6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passF_w_ab_1x25e6.log 2>&1
rc=$?; echo "gemm ab 1x2.5e7 rc=$rc"; grep -E "parity|median" $O/passF_w_ab_1x25e6.log
exit $rc
