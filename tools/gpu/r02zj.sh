#!/bin/bash
# round 2 re-entry: pass F with the tile y prefetched at the tile start
set -o pipefail
mkdir -p gpurun_out/r02zj /tmp/mb
O=gpurun_out/r02zj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nuts.py -m gpu -q -x --timeout 300 --timeout-method thread -k "regression_lpgrad or prior_lpgrad or placement or reproducible or fulldata or linear_regression_closed or logistic_matches" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/sw 2>/dev/null || exit 5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- /tmp/mb/sw 2000000 8 1000 5 64 > $O/micro.log 2>&1 || exit 3
grep -E "v5" $O/micro.log
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -3 $O/stats.csv
