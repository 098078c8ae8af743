#!/bin/bash
# round 2 re-entry: the full-size shard-sum property test, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/r02zx
O=gpurun_out/r02zx
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 240 --timeout-method thread -k "fullsize" > $O/pytest_fullsize.log 2>&1
rc=$?; echo "fullsize rc=$rc"; tail -3 $O/pytest_fullsize.log; [ $rc -le 1 ] || exit 2
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
