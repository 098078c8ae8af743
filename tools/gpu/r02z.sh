#!/bin/bash
# round 2 re-entry: the restored tree on a fresh box -- GPU parity suite, smoke, default bench line
set -o pipefail
mkdir -p gpurun_out/r02z
O=gpurun_out/r02z
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit 2
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 4
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('N1', d['value'], d['ms_per_step'], d['ess_per_sec'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['combine'])"
