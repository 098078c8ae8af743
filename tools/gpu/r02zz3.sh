#!/bin/bash
# round 2 re-entry: pass B with 128-column blocks (all 64 chains per wave, 3-deep ring of 48 KB
# stages) vs 64-column blocks: same-box A/B, after the C = 64 parity tests of the default build
set -o pipefail
mkdir -p gpurun_out/r02zz3 /tmp/mb
O=gpurun_out/r02zz3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nuts.py -m gpu -q -x --timeout 300 --timeout-method thread -k "regression_lpgrad or prior_lpgrad or placement or reproducible or fulldata" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DG5_BJB=128 -DG5_BNS=3 tools/sweep_micro.hip -o /tmp/mb/b128 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/b64 2>/dev/null || exit 5
for v in b128 b64 b128 b64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- /tmp/mb/$v 2000000 8 1000 5 64 > $O/micro_$v.log 2>&1 || exit 3
  echo "$v $(grep -E 'v5 flops' $O/micro_$v.log)"
  python3 tools/rocpd_summary.py stats $O/prof_$v/run_results.db > $O/stats_$v.csv 2>&1; sed -n 2,3p $O/stats_$v.csv
done
