#!/bin/bash
# round 3, call l: 8-schools fused kernel with the schools' data in registers, leapfrog counts in
# registers and the stack scalars in LDS: the NUTS GPU tests (twin, packed-vs-unpacked bitwise,
# exact moments) and configs[1] (4096 chains, Stan defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_kernels.py -k "schools or transition or nuts or moments or packed" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 300 python3 -u tools/bench_schools.py > $O/schools.json 2> $O/schools.err
rc=$?; echo "schools rc=$rc"; cat $O/schools.json | cut -c1-600
