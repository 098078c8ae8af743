#!/bin/bash
# round 2 re-entry: k_sweepe residual without row masks on full sub-tiles (SE_FAST) -- parity,
# then a same-box A/B
set -o pipefail
mkdir -p gpurun_out/r02zz2 /tmp/mb
O=gpurun_out/r02zz2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nuts.py -m gpu -q -x --timeout 240 --timeout-method thread -k "regression_lpgrad or prior_lpgrad or placement or fullsize or transition_matches_oracle_logistic or reproducible" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DSE_FAST=1 tools/sweep_micro.hip -o /tmp/mb/f1 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DSE_FAST=0 tools/sweep_micro.hip -o /tmp/mb/f0 2>/dev/null || exit 5
for v in f1 f0 f1 f0 f1 f0; do
  STARK_SWEEPM=e timeout -k 10 120 /tmp/mb/$v 12500000 8 100 10 16 > $O/micro_$v.log 2>&1 || exit 3
  echo "$v $(grep -E '^v4e  ' $O/micro_$v.log)"
done
