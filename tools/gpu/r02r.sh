#!/bin/bash
# round 2, call r: the LDS-staged NUTS step vs the global-memory one at one shard per GPU (the
# per-rank workload of the 8-GPU run), kernel traces; then the NUTS parity tests
set -o pipefail
mkdir -p gpurun_out/r02r
O=gpurun_out/r02r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in global; do
  STARK_NUTS_STEP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --rows 1.25e7 --shards 1 --steps 300 --warmup 20 --no-cpu-baseline --no-accuracy > $O/bench_1shard_$v.json 2> $O/bench_1shard_$v.err || exit 2
  python3 tools/rocpd_summary.py stats $O/prof_$v/run_results.db > $O/stats_$v.csv 2>&1
  head -4 $O/stats_$v.csv
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_nuts.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_nuts.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest_nuts.log
