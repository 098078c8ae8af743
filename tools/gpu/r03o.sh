#!/bin/bash
# round 3, call o: NUTS tests after the cold-path outlining; 8 schools (product, and chains_per_wave
# 2 at two waves per SIMD from an -DSTK_FUSED_MINW2 build); full-data pass F with residual v3 and
# static chain tiles vs the previous tree (kernel trace, same box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools.json 2> $O/schools.err || exit 5
cut -c1-110 $O/schools.json
STARK_HIP_LIB=$GRAFT_REPO_ROOT/tools/_bin/exp_minw2/libstark_hip.so timeout -k 10 200 python3 -u tools/bench_schools.py --chains-per-wave 2 > $O/schools_cpw2_minw2.json 2> $O/schools_cpw2_minw2.err || exit 6
cut -c1-110 $O/schools_cpw2_minw2.json
for v in base new; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/tools/_bin/base_lib/libstark_hip.so; else L=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so; fi
  STARK_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fd_$v -o run -- python3 tools/bench_fulldata.py --rows-per-gpu 4e6 --steps 20 > $O/fd_$v.json 2> $O/fd_$v.err || exit 7
  python3 tools/rocpd_summary.py stats $O/fd_$v/run_results.db > $O/fd_${v}_stats.csv 2>&1; grep -E "gemm" $O/fd_${v}_stats.csv
done
