#!/bin/bash
# round 2, call f: packed-schools bitwise test, combine inverse v4, config-2 variants
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nuts.py tests/test_gpu_kernels.py -m gpu -q --timeout 250 --timeout-method thread -k "schools or combine" > $O/r02f_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 3
timeout -k 10 120 python3 tools/combine_bench.py > $O/r02f_combine.json 2>&1 || exit 6
for v in "4 1" "4 2" "2 1" "2 2" "1 2"; do set -- $v
  STARK_FUSED_CPW=$1 STARK_FUSED_MINW=$2 timeout -k 10 120 python3 tools/bench_schools.py > $O/r02f_schools_cpw$1_minw$2.json 2>&1 || exit 5
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/r02f_prof -o combine -- python3 $GRAFT_REPO_ROOT/tools/combine_bench.py > $GRAFT_REPO_ROOT/$O/r02f_prof_combine.log 2>&1
echo "prof rc=$?"
