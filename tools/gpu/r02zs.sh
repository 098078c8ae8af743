#!/bin/bash
# round 2 re-entry: combine GEMM vector loaders + k_sweepe beta-image padding: parity, then
# same-box A/B (SE_BPAD 0 vs 2) of the sweep and the combine kernel split
set -o pipefail
mkdir -p gpurun_out/r02zs /tmp/mb
O=gpurun_out/r02zs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_consensus.py tests/test_gpu_nuts.py -m gpu -q -x --timeout 300 --timeout-method thread -k "combine or consensus or contract or regression_lpgrad or prior_lpgrad or placement or transition_matches_oracle_logistic" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DSE_BPAD=0 tools/sweep_micro.hip -o /tmp/mb/p0 2>/dev/null || exit 5
hipcc -O3 --offload-arch=gfx950 -std=c++17 -DSE_BPAD=2 tools/sweep_micro.hip -o /tmp/mb/p2 2>/dev/null || exit 5
for v in p0 p2 p0 p2; do
  STARK_SWEEPM=e timeout -k 10 120 /tmp/mb/$v 12500000 8 100 10 16 > $O/micro_$v.log 2>&1 || exit 3
  echo "$v $(grep -E '^v4e  ' $O/micro_$v.log)"
done
hipcc -O3 --offload-arch=gfx950 -I stark_amd/csrc tools/mgemm_micro.hip -o /tmp/mb/m 2>/dev/null || exit 5
timeout -k 5 60 /tmp/mb/m > $O/mgemm_micro.log 2>&1 || exit 6
cat $O/mgemm_micro.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/combine_bench.py > $O/combine.json 2> $O/combine.err || exit 7
cat $O/combine.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -10 $O/stats.csv
