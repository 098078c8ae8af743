#!/bin/bash
# round 3 (re-entry), call e: k_sweepe A/B (residual v2 + early release vs round-2 kernel) at the
# bench geometry; the full GPU suite; smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 240 tools/_bin/sweepe_ab 12500000 8 3 8 > $O/sweepe_ab.log 2>&1
rc=$?; echo "sweepe_ab rc=$rc"; grep -E "parity|median" $O/sweepe_ab.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
