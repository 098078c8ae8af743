#!/bin/bash
# round 4, call s: r04r's A/B again with the committed kernel and k_sweepe launched with their
# own LDS size (r04r gave them the new, smaller one)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 240 tools/_bin/sweep16_ab 12500000 8 5 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "parity|median" $O/ab_d100.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 3 10 50 2 > $O/ab_d50.log 2>&1
rc=$?; echo "ab d50 rc=$rc"; grep -E "parity|median" $O/ab_d50.log
