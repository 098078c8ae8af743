#!/bin/bash
# round 5, call l: stamped 8-schools breakdown after the single end_transition site; k_sweep16 DPP
# single-register VALU tail A/B repeated on another box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 200 python3 -u tools/schools_stamps.py run > $O/schools_stamps.json 2> $O/schools_stamps.err
rc=$?; echo "stamps rc=$rc"; cat $O/schools_stamps.json; [ $rc -eq 0 ] || exit 4
timeout -k 10 300 tools/_bin/sweep16_ab 12500000 8 7 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "median" $O/ab_d100.log
