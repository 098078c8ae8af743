#!/bin/bash
# round 3, call y: 8 schools with normal_lpdf's inverse sigma computed once per launch (Stan
# Math 2.19's arithmetic; no f64 division per leapfrog) in the in-tree library -- NUTS and kernel
# tests, then alternating against the r03w winner (dpp)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 4
lib() { case $1 in dpp*) echo $GRAFT_REPO_ROOT/tools/_bin/dpp_lib/libstark_hip.so;; *) echo $GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; esac; }
for v in dpp isig dpp2 isig2 dpp3 isig3; do
  STARK_HIP_LIB=$(lib $v) timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  echo $v $(cut -c1-120 $O/schools_$v.json)
done
