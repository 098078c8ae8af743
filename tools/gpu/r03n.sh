#!/bin/bash
# round 3, call n: transition-end math (Box-Muller, dual averaging) out of line in the NUTS state
# machine: NUTS GPU tests and 8 schools x 4096 chains
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for i in 1 2; do timeout -k 10 300 python3 -u tools/bench_schools.py > $O/schools$i.json 2> $O/schools$i.err || exit 5; cut -c1-120 $O/schools$i.json; done
