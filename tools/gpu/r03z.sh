#!/bin/bash
# round 3, call z: 8 schools, 2 chains per wave at two waves per SIMD (STK_FUSED_MINW2: 256
# registers, 15 spilled, after the round-3 register cuts) vs the default 4 chains per wave
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03z
mkdir -p $O
M2=$GRAFT_REPO_ROOT/tools/_bin/minw2/libstark_hip.so
STARK_HIP_LIB=$M2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py -k "schools or packed" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for v in cpw4 m2 cpw4b m2b; do
  case $v in cpw4*) A="";; *) A="--chains-per-wave 2";; esac
  case $v in cpw4*) L=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; *) L=$M2;; esac
  STARK_HIP_LIB=$L timeout -k 10 200 python3 -u tools/bench_schools.py $A > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  echo $v $(cut -c1-120 $O/schools_$v.json)
done
