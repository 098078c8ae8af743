#!/bin/bash
# round 5, call g: pass F with 128-row tiles shared by 8 waves (one block per CU; 2 and 3 stages)
# against the product (configs[4]'s shape: 8 x 2e6 rows, d = 1000, 64 chains)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_w128_ab.log 2>&1
rc=$?; echo "gemm ab rc=$rc"; grep -E "parity|median" $O/passF_w128_ab.log
