#!/bin/bash
# round 4, call z: k_sweep16 with the chunk count per shard (256, 512 = the library, 1024)
# at d = 100 logistic, 5 interleaved rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z2
mkdir -p $O
timeout -k 10 300 tools/_bin/sweep16_ab 12500000 8 5 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "parity|median" $O/ab_d100.log
