#!/bin/bash
# round 5, call ag: HBM bytes per launch of the 64-chain GEMM passes (FETCH_SIZE and WRITE_SIZE in
# separate passes over the gemm_ab harness at configs[4]'s shape) against their algorithmic bytes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_gemm_traffic.py $O/pmc_fetch/pmc_counter_collection.csv $O/pmc_write/pmc_counter_collection.csv --rows-per-shard 2000000 --shards 8 --d 1000 --json $O/gemm_traffic.json
