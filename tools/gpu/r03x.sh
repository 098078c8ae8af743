#!/bin/bash
# round 3, call x: 8 schools -- the r03w winner (cold scalars + row_newbcast + bound_ctrl DPP,
# dpp) vs that plus an opaque Philox seed per call (seed: the round-key schedule no longer
# hoisted and spilled into VGPR lanes), alternating; NUTS + kernel tests on seed first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03x
mkdir -p $O
B=$GRAFT_REPO_ROOT/tools/_bin
lib() { case $1 in base*) echo $GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; dpp*) echo $B/dpp_lib/libstark_hip.so;; *) echo $B/seed_lib/libstark_hip.so;; esac; }
STARK_HIP_LIB=$(lib seed) timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_kernels.py > $O/pytest_seed.log 2>&1
rc=$?; echo "pytest seed rc=$rc"; tail -1 $O/pytest_seed.log; [ $rc -eq 0 ] || exit 4
for v in dpp seed dpp2 seed2 dpp3 seed3; do
  STARK_HIP_LIB=$(lib $v) timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  echo $v $(cut -c1-120 $O/schools_$v.json)
done
