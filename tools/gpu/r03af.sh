#!/bin/bash
# round 3, call af: the SPD inverse's 16 x 16 pivot steps with DPP row broadcasts (one
# ds_bpermute per pivot instead of six) -- kernel + consensus tests, then the combine under a
# kernel trace (k_spd_inverse was 46 us per call in r03ae)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/combine_bench.py > $O/combine.json 2> $O/combine.err || exit 5
cut -c1-600 $O/combine.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; grep -E "spd|mgemm|row_stats" $O/stats.csv
rm -rf $O/prof
