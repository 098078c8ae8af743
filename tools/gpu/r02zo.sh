#!/bin/bash
# (run from a git checkout: the old sweep.hip comes from history)
# round 2 re-entry: same-box A/B of the C = 64 GEMM passes, bf842b3 (before the rework) vs this tree
set -o pipefail
mkdir -p gpurun_out/r02zo /tmp/mb /tmp/ab/stark_amd/csrc /tmp/ab/tools /tmp/ab/include
O=gpurun_out/r02zo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
cp include/*.h /tmp/ab/include/ && cp stark_amd/csrc/*.h stark_amd/csrc/datagen.hip /tmp/ab/stark_amd/csrc/ && git show bf842b3:stark_amd/csrc/sweep.hip > /tmp/ab/stark_amd/csrc/sweep.hip && cp tools/sweep_micro.hip /tmp/ab/tools/ || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 /tmp/ab/tools/sweep_micro.hip -o /tmp/mb/old 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/new 2>/dev/null || exit 5
for v in old new old new; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- /tmp/mb/$v 2000000 8 1000 5 64 > $O/micro_$v.log 2>&1 || exit 3
  echo "$v $(grep -E 'v5 flops' $O/micro_$v.log)"
  python3 tools/rocpd_summary.py stats $O/prof_$v/run_results.db > $O/stats_$v.csv 2>&1; sed -n 2,3p $O/stats_$v.csv
done
