#!/bin/bash
# round 2 re-entry: pass F with 16-column stages in a 4-deep ring (library default for this
# call): parity, then same-box A/B against 32-column stages in a double buffer
set -o pipefail
mkdir -p gpurun_out/r02zy /tmp/mb
O=gpurun_out/r02zy
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nuts.py -m gpu -q -x --timeout 300 --timeout-method thread -k "regression_lpgrad or prior_lpgrad or placement or reproducible or fulldata" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DG5_FKC=16 -DG5_FS=4 tools/sweep_micro.hip -o /tmp/mb/k16 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DG5_FKC=32 -DG5_FS=2 tools/sweep_micro.hip -o /tmp/mb/k32 2>/dev/null || exit 5
for v in k16 k32 k16 k32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- /tmp/mb/$v 2000000 8 1000 5 64 > $O/micro_$v.log 2>&1 || exit 3
  echo "$v $(grep -E 'v5 flops' $O/micro_$v.log)"
  python3 tools/rocpd_summary.py stats $O/prof_$v/run_results.db > $O/stats_$v.csv 2>&1; sed -n 2,3p $O/stats_$v.csv
done
