#!/bin/bash
# round 5, call as: the split pass F with alpha re-read at the park (1 VGPR spilled instead of 4)
# (A/B at both shapes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05as
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_split_8x2e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-split-alpha|median" $O/passF_split_8x2e6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passF_split_1x25e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-split-alpha|median" $O/passF_split_1x25e6.log
exit $rc
