#!/bin/bash
# Consensus moments at the headline scale (N = 1e8, d = 100, 8 shards x 16 chains): per-shard
# and consensus z against the generating parameters with 450 kept draws per chain.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 780 python3 -u tools/consensus_check.py --rows 1e8 --d 100 --warmup 150 --samples 450 > gpurun_out/consensus_1e8.log 2>&1
rc=$?; echo "consensus rc=$rc"; tail -25 gpurun_out/consensus_1e8.log
exit $rc
