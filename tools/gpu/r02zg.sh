#!/bin/bash
# round 2 re-entry: per-kernel split of the C = 64 two-pass GEMM sweep (configs[4] geometry)
set -o pipefail
mkdir -p gpurun_out/r02zg /tmp/mb
O=gpurun_out/r02zg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/sw 2>/dev/null || exit 5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- /tmp/mb/sw 2000000 8 1000 5 64 > $O/micro.log 2>&1 || exit 2
grep -E "v5|sweep" $O/micro.log
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -8 $O/stats.csv
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc -o pmc --output-format csv -- /tmp/mb/sw 2000000 8 1000 2 64 > $O/pmc.log 2>&1 || exit 3
ls -R $O/pmc | head
