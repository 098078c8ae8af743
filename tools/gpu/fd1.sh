#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fulldata" > gpurun_out/pytest_fd.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_fd.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_fulldata.py > gpurun_out/bench_fd.log 2>&1
rc=$?; echo "bench fd rc=$rc"; tail -3 gpurun_out/bench_fd.log
