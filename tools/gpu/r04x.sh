#!/bin/bash
# round 4, call x: final validation of the tree -- the full GPU suite, smoke, and the default bench
# line as the driver runs it (now with the configs[2] / configs[4] throughput sub-records)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04x
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 480 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 5
fi
T0=$(date +%s)
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc, $(( $(date +%s) - T0 )) s"; [ $rc -eq 0 ] || exit 8
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; o=d['other_configs'] or {}; print('bench', d['value'], d['ess_per_sec'], r['frac'], r['avg_launch_ms'], (d.get('configs1_schools') or {}).get('value'), (d.get('ess_second_criterion') or {}).get('ess_per_sec')); print('c2', {k: v for k, v in (o.get('configs2_linear') or {}).items() if k in ('value', 'ms_per_step', 'error')}); print('c4', {k: v for k, v in (o.get('configs4_fulldata') or {}).items() if k in ('value', 'ms_per_step', 'error')})"
