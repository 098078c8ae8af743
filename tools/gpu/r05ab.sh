#!/bin/bash
# round 5, call ab: pass F with the next stage DMA issued right after the barrier (before the epilogue part and y loads)
# and the same bytes as one sequential stream, against the product (configs[4]'s shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_early_ab.log 2>&1
rc=$?; echo "gemm ablations rc=$rc"; grep -E "parity|median" $O/passF_early_ab.log
exit $rc
