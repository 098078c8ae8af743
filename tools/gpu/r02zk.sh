#!/bin/bash
# round 2 re-entry: pass F epilogue with 1 / 2 / 4 residuals in flight (G5_EU)
set -o pipefail
mkdir -p gpurun_out/r02zk /tmp/mb
O=gpurun_out/r02zk
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for u in 1 2 4; do
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -DG5_EU=$u tools/sweep_micro.hip -o /tmp/mb/sw$u 2>/dev/null || exit 5
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof$u -o run -- /tmp/mb/sw$u 2000000 8 1000 5 64 > $O/micro$u.log 2>&1 || exit 3
  echo "EU=$u $(grep -E 'v5 flops' $O/micro$u.log)"
  python3 tools/rocpd_summary.py stats $O/prof$u/run_results.db > $O/stats$u.csv 2>&1; sed -n 2,3p $O/stats$u.csv
done
