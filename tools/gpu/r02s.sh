#!/bin/bash
# round 2, call s: one shard per GPU after the NUTS-step inlining fix and the 16-wave reduce;
# 8-schools config 2 after the inlining fix; GPU tests of the touched kernels
set -o pipefail
mkdir -p gpurun_out/r02s
O=gpurun_out/r02s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --rows 1.25e7 --shards 1 --steps 300 --warmup 20 --no-cpu-baseline --no-accuracy > $O/bench_1shard.json 2> $O/bench_1shard.err || exit 2
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats_1shard.csv 2>&1; head -4 $O/stats_1shard.csv
timeout -k 10 300 python3 tools/bench_schools.py > $O/schools.json 2> $O/schools.err || exit 3
tail -c 400 $O/schools.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_nuts.py tests/test_gpu_kernels.py tests/test_gpu_consensus.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest.log
