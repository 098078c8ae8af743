#!/bin/bash
# round 5, call e: pass F (k_gemm_fwd, configs[4]'s shape: 8 x 2e6 rows, d = 1000, 64 chains) with
# the tile's R stores deferred to the next stage's top (no tile-end vmcnt(0)) against the product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_defer_ab.log 2>&1
rc=$?; echo "gemm ab rc=$rc"; grep -E "parity|median" $O/passF_defer_ab.log
