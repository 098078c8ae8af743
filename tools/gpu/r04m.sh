#!/bin/bash
# round 4, call m: k_sweep16 wave-priority variants A/B at d = 100.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 5 8 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "d100 rc=$rc"; grep -E "parity|median" $O/ab_d100.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 5 8 100 3 > $O/ab_d100_2.log 2>&1
rc=$?; echo "d100 (2) rc=$rc"; grep median $O/ab_d100_2.log
