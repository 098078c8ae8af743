#!/bin/bash
# round 2 re-entry: PMC of the reworked full-data GEMM passes (MFMA busy, waits, clock)
set -o pipefail
mkdir -p gpurun_out/r02zz9 /tmp/mb
O=gpurun_out/r02zz9
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/sw 2>/dev/null || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc -o pmc --output-format csv -- /tmp/mb/sw 2000000 8 1000 2 64 > $O/pmc.log 2>&1 || exit 3
echo pmc ok
