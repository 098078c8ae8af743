#!/bin/bash
# round 5, call v: pass B at 4 waves with 2-4 column tiles per wave, 8-16-row stages, 2-4 stage rings
# fewer rows per stage, against the product, at configs[4]'s shape and at bench's
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passB_ab_8x2e6.log 2>&1
rc=$?; echo "gemm ab 8x2e6 rc=$rc"; grep -E "parity|median" $O/passB_ab_8x2e6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passB_ab_1x25e6.log 2>&1
rc=$?; echo "gemm ab 1x2.5e7 rc=$rc"; grep -E "parity|median" $O/passB_ab_1x25e6.log
exit $rc
