#!/bin/bash
# round 2 re-entry: 4-wide vector loaders in the combine GEMMs -- combine parity tests, micro, kernel split
set -o pipefail
mkdir -p gpurun_out/r02zr
O=gpurun_out/r02zr
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_consensus.py -m gpu -q -x --timeout 200 --timeout-method thread -k "combine or consensus or reduce or contract or singular or inverse" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log; [ $rc -le 1 ] || exit 2
mkdir -p /tmp/mb && hipcc -O3 --offload-arch=gfx950 -I stark_amd/csrc tools/mgemm_micro.hip -o /tmp/mb/m 2>/dev/null || exit 5
timeout -k 5 60 /tmp/mb/m > $O/micro.log 2>&1 || exit 6
cat $O/micro.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/combine_bench.py > $O/combine.json 2> $O/combine.err || exit 3
cat $O/combine.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -12 $O/stats.csv
