#!/bin/bash
# round 5, call f: the whole GPU suite (new: bench --gpus 2 rehearsal, duplicated-row singular
# combine, pass F long-chunk parity, 8-schools divergence rate vs the oracle twin) and smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v -m gpu --timeout 500 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
