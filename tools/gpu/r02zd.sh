#!/bin/bash
# round 2 re-entry: the fp64 MFMA ceiling micro with and without the VGPR-form MFMA codegen
# (-mllvm -amdgpu-mfma-vgpr-form: the default build moves every accumulator AGPR<->VGPR per loop trip)
set -o pipefail
mkdir -p gpurun_out/r02zd /tmp/mb
O=gpurun_out/r02zd
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_ceiling.hip -o /tmp/mb/c_agpr 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form tools/mfma_ceiling.hip -o /tmp/mb/c_vgpr 2>/dev/null || exit 5
echo "== default codegen"; timeout -k 5 120 /tmp/mb/c_agpr 20000 | tee $O/ceiling_default.log || exit 6
echo "== vgpr-form codegen"; timeout -k 5 120 /tmp/mb/c_vgpr 20000 | tee $O/ceiling_vgprform.log || exit 6
