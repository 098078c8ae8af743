#!/bin/bash
# round 2 re-entry: MFMA/VALU overlap and the sweep variants under the clean (VGPR-form) MFMA codegen
set -o pipefail
mkdir -p gpurun_out/r02ze /tmp/mb
O=gpurun_out/r02ze
F="-mllvm -amdgpu-mfma-vgpr-form"
hipcc -O3 --offload-arch=gfx950 $F tools/mfma_overlap.hip -o /tmp/mb/ov 2>/dev/null || exit 5
timeout -k 5 60 /tmp/mb/ov > $O/overlap_vgprform.log 2>&1 || exit 6
cat $O/overlap_vgprform.log
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o /tmp/mb/sw 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 $F tools/sweep_micro.hip -o /tmp/mb/swv 2>/dev/null || exit 5
for v in e q x; do
  STARK_SWEEPM=$v timeout -k 10 120 /tmp/mb/sw 12500000 8 100 10 16 > $O/micro_$v.log 2>&1 || exit 2
  echo "default $v: $(tail -1 $O/micro_$v.log)"
  STARK_SWEEPM=$v timeout -k 10 120 /tmp/mb/swv 12500000 8 100 10 16 > $O/micro_${v}_vgprform.log 2>&1 || exit 2
  echo "vgprform $v: $(tail -1 $O/micro_${v}_vgprform.log)"
done
