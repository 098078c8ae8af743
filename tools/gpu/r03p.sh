#!/bin/bash
# round 3, call p: NUTS momentum with one sincos (NUTS tests, 8 schools); pass F with residual v3
# only (the round-2 loop kept) vs the previous tree, kernel trace on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for i in 1 2; do timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools$i.json 2> $O/schools$i.err || exit 5; cut -c1-110 $O/schools$i.json; done
for v in base new base2 new2; do
  case $v in base*) L=$GRAFT_REPO_ROOT/tools/_bin/base_lib/libstark_hip.so;; *) L=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; esac
  STARK_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fd_$v -o run -- python3 tools/bench_fulldata.py --rows-per-gpu 4e6 --steps 20 > $O/fd_$v.json 2> $O/fd_$v.err || exit 7
  python3 tools/rocpd_summary.py stats $O/fd_$v/run_results.db > $O/fd_${v}_stats.csv 2>&1; echo $v; grep -E "gemm_fwd" $O/fd_${v}_stats.csv
done
