#!/bin/bash
# round 3, call r: v_rcp_f64's accuracy (is the Newton step needed?), and k_sweepe with the
# residual's Newton step dropped (RV 4) and a degree-3 exp (RV 5), A/B at the bench geometry
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 60 tools/_bin/rcp_acc > $O/rcp_acc.log 2>&1; rc=$?; cat $O/rcp_acc.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 tools/_bin/sweepe_ab 12500000 8 4 8 > $O/sweepe_ab.log 2>&1
rc=$?; echo "sweepe_ab rc=$rc"; grep -E "parity|median" $O/sweepe_ab.log
