#!/bin/bash
# round 5, call ag: HBM bytes per launch of the 64-chain GEMM passes (FETCH_SIZE and WRITE_SIZE in
# separate passes over the gemm_ab harness at configs[4]'s shape) against their algorithmic bytes;
# first the 64-chain parity tests at the largest d
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "4096-64 or 2049-64" > $O/pytest_maxd.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_maxd.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_gemm_traffic.py $O/pmc_fetch/pmc_counter_collection.csv $O/pmc_write/pmc_counter_collection.csv --rows-per-shard 2000000 --shards 8 --d 1000 --json $O/gemm_traffic.json
