#!/bin/bash
# round 2, call m: block (4-pivot) SPD inverse -- combine parity tests, latency, kernel split
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_consensus.py -m gpu -q --timeout 250 --timeout-method thread > $O/r02m_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/r02m_pytest.log; [ $rc -le 1 ] || exit 3
timeout -k 10 120 python3 tools/combine_bench.py > $O/r02m_combine.json 2>&1 || exit 4
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/r02m_prof -o combine --output-format csv -- python3 tools/combine_bench.py > $O/r02m_prof_combine.log 2>&1
echo "prof rc=$?"
