#!/bin/bash
# round 3, call s: v_rcp_f64 accuracy; k_sweepe residual without the Newton step (RV 4) / with a
# degree-3 exp (RV 5) A/B; the NUTS state machine's cold paths out of line (fused kernel: scalar
# state in LDS): NUTS GPU tests and 8 schools x 4096 chains
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 60 tools/_bin/rcp_acc > $O/rcp_acc.log 2>&1; rc=$?; cat $O/rcp_acc.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 tools/_bin/sweepe_ab 12500000 8 4 8 > $O/sweepe_ab.log 2>&1
rc=$?; echo "sweepe_ab rc=$rc"; grep -E "parity|median" $O/sweepe_ab.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for i in 1 2; do timeout -k 10 200 python3 -u tools/bench_schools.py > $O/schools$i.json 2> $O/schools$i.err || exit 5; cut -c1-110 $O/schools$i.json; done
