#!/bin/bash
# round 2 re-entry: k_sweepe variants (EARLY: all slot reads before the forward MFMAs)
set -o pipefail
mkdir -p gpurun_out/r02zf /tmp/mb
O=gpurun_out/r02zf
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/sw 2>/dev/null || exit 5
STARK_SWEEPM=e timeout -k 10 120 /tmp/mb/sw 12500000 8 100 10 16 > $O/micro_e.log 2>&1 || exit 2
grep -E "v4e|sweep" $O/micro_e.log
