#!/bin/bash
# round 2 final closing check (after the per-device LDS attribute change): smoke, the default bench line
# under a kernel trace (its timed window checked against the trace), the driver-shaped line
set -o pipefail
mkdir -p gpurun_out/r02zz12
O=gpurun_out/r02zz12
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/bench.json 2> $O/bench.err || exit 4
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweepe --bench-json $O/bench.json --json $O/window.json || exit 5
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -5 $O/stats.csv
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ess_per_sec'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'], d['combine']['gpu_ms'])"
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 6
python3 -c "import json; d=json.loads(open('$O/bench_steps20.json').read().strip().splitlines()[-1]); print('steps20', d['value'], d['ess_per_sec'], d['roofline']['frac'])"
