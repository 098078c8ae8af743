#!/bin/bash
# round 5, call af: pass F with the next stage DMA spread over the k-steps
# and the same bytes as one sequential stream, against the product (configs[4]'s shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_spread_ab.log 2>&1
rc=$?; echo "gemm ablations rc=$rc"; grep -E "parity|median" $O/passF_spread_ab.log
exit $rc
