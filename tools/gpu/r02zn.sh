#!/bin/bash
# round 2 re-entry: A/B on one box -- GEMM stage-ring barriers raw (s_barrier) vs __syncthreads()
set -o pipefail
mkdir -p gpurun_out/r02zn /tmp/mb
O=gpurun_out/r02zn
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DG5_RAWBAR=1 tools/sweep_micro.hip -o /tmp/mb/raw 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DG5_RAWBAR=0 tools/sweep_micro.hip -o /tmp/mb/sync 2>/dev/null || exit 5
for v in raw sync raw sync; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- /tmp/mb/$v 2000000 8 1000 5 64 > $O/micro_$v.log 2>&1 || exit 3
  echo "$v $(grep -E 'v5 flops' $O/micro_$v.log)"
  python3 tools/rocpd_summary.py stats $O/prof_$v/run_results.db > $O/stats_$v.csv 2>&1; sed -n 2,3p $O/stats_$v.csv
done
