#!/bin/bash
# round 2, re-entry: MFMA combine GEMMs: combine parity tests, then the combine's kernel split
set -o pipefail
mkdir -p gpurun_out/r02za
O=gpurun_out/r02za
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_consensus.py -m gpu -q -x --timeout 200 --timeout-method thread -k "combine or consensus or reduce or contract" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/combine_bench.py > $O/combine.json 2> $O/combine.err || exit 3
cat $O/combine.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -12 $O/stats.csv
