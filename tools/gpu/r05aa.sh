#!/bin/bash
# round 5, call aa: where pass F's X stage stream loses time -- X stages from an L2-resident tile,
# and the same bytes as one sequential stream, against the product (configs[4]'s shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aa
mkdir -p $O
GEMM_AB_ABL=1 timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_xstream_ablations.log 2>&1
rc=$?; echo "gemm ablations rc=$rc"; grep -E "median" $O/passF_xstream_ablations.log
exit $rc
