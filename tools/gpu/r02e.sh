#!/bin/bash
# round 2, call e: packed 8-schools chains (4 per wave) -- parity, config-2 bench at CPW 4 and 1,
# rocprof; combine inverse v3 latency
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nuts.py tests/test_gpu_kernels.py tests/test_gpu_consensus.py -m gpu -q --timeout 200 --timeout-method thread -k "schools or combine or stark or driver" > $O/r02e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 3
timeout -k 10 120 python3 tools/bench_schools.py > $O/r02e_schools_cpw4.json 2>&1 || exit 4
STARK_FUSED_CPW=1 timeout -k 10 120 python3 tools/bench_schools.py > $O/r02e_schools_cpw1.json 2>&1 || exit 5
timeout -k 10 120 python3 tools/combine_bench.py > $O/r02e_combine.json 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/r02e_prof -o schools -- python3 $GRAFT_REPO_ROOT/tools/bench_schools.py > $GRAFT_REPO_ROOT/$O/r02e_prof_schools.log 2>&1 || exit 7
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/r02e_prof -o combine -- python3 $GRAFT_REPO_ROOT/tools/combine_bench.py > $GRAFT_REPO_ROOT/$O/r02e_prof_combine.log 2>&1
echo "prof rc=$?"
