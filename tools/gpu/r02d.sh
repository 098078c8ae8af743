#!/bin/bash
# round 2, call d: combine v2 (split-K, register inverse) -- parity tests, latency, rocprof kernel split
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_consensus.py tests/test_gpu_nuts.py -m gpu -q --timeout 200 --timeout-method thread -k "combine or consensus or driver or stark" > $O/r02d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 3
timeout -k 10 120 python3 tools/combine_bench.py > $O/r02d_combine.json 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/r02d_prof -o combine -- python3 $GRAFT_REPO_ROOT/tools/combine_bench.py > $GRAFT_REPO_ROOT/$O/r02d_prof.log 2>&1
echo "prof rc=$?"
