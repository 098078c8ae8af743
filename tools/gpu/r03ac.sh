#!/bin/bash
# round 3, call ac: configs[2]'s sweep shape (linear, d = 50, 16 chains): the product k_sweepm
# vs k_sweepe instantiated for d = 50 (tools/sweepe_d50.hip), then the config-2 PMC (r03ab)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 200 tools/_bin/sweepe_d50 1250000 8 5 50 > $O/sweepe_d50.log 2>&1
rc=$?; echo "sweepe_d50 rc=$rc"; grep -E "parity|median|rows" $O/sweepe_d50.log; [ $rc -eq 0 ] || exit 3
bash tools/gpu/r03ab.sh
