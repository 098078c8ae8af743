#!/bin/bash
# round 4, call l: validation of the tree after the sweep and 8-schools changes -- the full GPU
# suite and smoke; the default bench line under a kernel trace (timed window vs trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 480 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 8
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweep16 --bench-json $O/bench.json --json $O/window.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -6 $O/stats.csv
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['bound'], r['frac'], r['avg_launch_ms'], r['traffic'], d['cpu_baseline'] and d['cpu_baseline'].get('value'), d['combine']['gpu_ms'], (d.get('configs1_schools') or {}).get('value'), (d.get('ess_second_criterion') or {}).get('ess_per_sec'))"
rm -rf $O/prof
