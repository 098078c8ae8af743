#!/bin/bash
# round 2 re-entry: k_sweepe under LLVM's AMDGPU scheduling strategies (same box A/B)
set -o pipefail
mkdir -p gpurun_out/r02zw /tmp/mb
O=gpurun_out/r02zw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/default 2>/dev/null || exit 5
for st in max-ilp max-memory-clause iterative-minreg; do
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-sched-strategy=$st tools/sweep_micro.hip -o /tmp/mb/$st 2>/dev/null || exit 5
done
for r in 1 2; do
  for v in default max-ilp max-memory-clause iterative-minreg; do
    STARK_SWEEPM=e timeout -k 10 120 /tmp/mb/$v 12500000 8 100 10 16 > $O/micro_${v}_$r.log 2>&1 || exit 3
    echo "$v $(grep -E '^v4e  ' $O/micro_${v}_$r.log)"
  done
done
