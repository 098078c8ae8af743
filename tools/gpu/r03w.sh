#!/bin/bash
# round 3, call w: 8 schools, libraries alternating on one box -- the committed one; the chain's
# cold scalars in memory (cold); + the segment broadcast by DPP row_newbcast (bcst); + DPP moves
# with bound_ctrl, no v_mov of the old value (dpp); + NutsArgs read from LDS at its uses
# (dpp_alds, STK_ARGS_LDS: fewer SGPR spills).  NUTS tests on the last two first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03w
mkdir -p $O
B=$GRAFT_REPO_ROOT/tools/_bin
lib() { case $1 in base*) echo $GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; cold*) echo $B/cold_lib/libstark_hip.so;;
        bcst*) echo $B/bcast_lib/libstark_hip.so;; dppa*) echo $B/dpp_alds/libstark_hip.so;; *) echo $B/dpp_lib/libstark_hip.so;; esac; }
for v in dpp dppa; do
  STARK_HIP_LIB=$(lib $v) timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || exit 4
done
for v in base cold bcst dpp dppa base2 cold2 bcst2 dpp2 dppa2; do
  STARK_HIP_LIB=$(lib $v) timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  echo $v $(cut -c1-120 $O/schools_$v.json)
done
