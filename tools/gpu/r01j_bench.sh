#!/bin/bash
# separate-lp combine test, default bench (block + joint consensus z), headline-scale consensus check.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "combine" -v --timeout 120 --timeout-method thread > gpurun_out/pytest_combine.log 2>&1
rc=$?; echo "pytest combine rc=$rc"; tail -3 gpurun_out/pytest_combine.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 660 python3 -u tools/consensus_check.py --rows 1e8 --d 100 --warmup 150 --samples 200 > gpurun_out/consensus_1e8_b.log 2>&1
rc=$?; echo "consensus rc=$rc"; tail -16 gpurun_out/consensus_1e8_b.log
exit $rc
