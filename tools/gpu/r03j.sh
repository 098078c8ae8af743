#!/bin/bash
# round 3, call j: combine tests (device draws read in place); the north_star accuracy check at
# N = 1e8 (8-shard consensus vs a full-data NUTS run of all rows, pooled batch MCSE, 250 and
# 1000 post-warmup draws per chain)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "combine" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 1000 python3 -u tools/fulldata_nuts_check.py --out $O/fulldata_nuts_check.json > $O/fdcheck.out 2> $O/fdcheck.err
rc=$?; echo "check rc=$rc"; tail -4 $O/fdcheck.err
