#!/bin/bash
# round 5, call y: pass F geometries (waves x row tiles per wave x stage columns x ring depth) against
# the product's 4w2r16k3s, at configs[4]'s shape and at bench's
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_geom_8x2e6.log 2>&1
rc=$?; echo "gemm ab 8x2e6 rc=$rc"; grep -E "parity|median" $O/passF_geom_8x2e6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passF_geom_1x25e6.log 2>&1
rc=$?; echo "gemm ab 1x2.5e7 rc=$rc"; grep -E "parity|median" $O/passF_geom_1x25e6.log
exit $rc
