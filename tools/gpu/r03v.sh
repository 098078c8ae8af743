#!/bin/bash
# round 3, call v: the NUTS chain's transition-end scalars and counters kept in memory (the
# fused kernel's LDS image) instead of registers -- NUTS tests on that library, then 8 schools
# A/B against the committed library, alternating, on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03v
mkdir -p $O
NEW=$GRAFT_REPO_ROOT/tools/_bin/cold_lib/libstark_hip.so
BASE=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so
STARK_HIP_LIB=$NEW timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for v in base new base2 new2 base3 new3; do
  case $v in base*) L=$BASE;; *) L=$NEW;; esac
  STARK_HIP_LIB=$L timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  echo $v $(cut -c1-120 $O/schools_$v.json)
done
