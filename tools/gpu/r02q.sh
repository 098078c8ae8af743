#!/bin/bash
# round 2, call q: the per-rank workload of the 8-GPU run (one 1.25e7-row shard) on one GPU,
# with a kernel trace: how much of a step is the sweep at one shard per GPU
set -o pipefail
mkdir -p gpurun_out/r02q
O=gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r02q/prof -o run -- python3 bench.py --rows 1.25e7 --shards 1 --steps 300 --warmup 20 --no-cpu-baseline --no-accuracy > $O/r02q/bench_1shard.json 2> $O/r02q/bench_1shard.err
echo "rc=$?"
tail -c 600 $O/r02q/bench_1shard.json
find $O/r02q/prof -name "*kernel_stats.csv" | head -3
