#!/bin/bash
# round 2, call h: fixed extended-criterion tests, combine profile, consensus diagnostics at
# N = 1e8 (Stan >= 2.23 criterion, 500 draws/chain), config-2 bench with roofline, headline bench
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts.py -m gpu -q --timeout 250 --timeout-method thread -k "extended" > $O/r02h_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 3
timeout -k 10 100 python3 tools/bench_schools.py > $O/r02h_schools.json 2>&1 || exit 4
timeout -k 10 120 tools/_bin/mfma_ceiling 20000 > $O/r02h_fp64_ceiling.log 2>&1 || exit 8
cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/r02h_prof -o combine -- python3 $GRAFT_REPO_ROOT/tools/combine_bench.py > $GRAFT_REPO_ROOT/$O/r02h_prof_combine.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/consensus_check.py --nuts-criterion stan2.23 --samples 500 --block 100 --out $O/r02h_consensus_check.jsonl > $O/r02h_consensus_check.log 2>&1 || exit 6
timeout -k 10 590 python3 bench.py --steps 20 --warmup 5 > $O/r02h_bench.json 2> $O/r02h_bench.err
echo "bench rc=$?"
