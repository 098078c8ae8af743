#!/bin/bash
# Headline-scale consensus check with the shard-level common-error diagnostics.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 680 python3 -u tools/consensus_check.py --rows 1e8 --d 100 --warmup 150 --samples 250 > gpurun_out/consensus_1e8_d.log 2>&1
rc=$?; echo "consensus rc=$rc"; tail -12 gpurun_out/consensus_1e8_d.log
exit $rc
