#!/bin/bash
# round 5, call ae: pass F with 8-column stages in 4-6 deep rings
# and the same bytes as one sequential stream, against the product (configs[4]'s shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_k8_ab.log 2>&1
rc=$?; echo "gemm ablations rc=$rc"; grep -E "parity|median" $O/passF_k8_ab.log
exit $rc
