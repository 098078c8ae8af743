#!/bin/bash
# round 2 re-entry: full GPU parity suite, smoke, driver-shaped bench, the default bench under a
# kernel trace (rocprof summary), full-data bench lines (configs[4] geometry)
set -o pipefail
mkdir -p gpurun_out/r02zp
O=gpurun_out/r02zp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 4
python3 -c "import json; d=json.loads(open('$O/bench_steps20.json').read().strip().splitlines()[-1]); print('N1 steps20', d['value'], d['ess_per_sec'], d['roofline']['frac'], d['combine']['gpu_ms'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run -- python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 5
python3 tools/rocpd_summary.py stats $O/prof_bench/run_results.db > $O/bench_kernel_stats.csv 2>&1; head -6 $O/bench_kernel_stats.csv
timeout -k 10 400 python3 tools/bench_fulldata.py --rows-per-gpu 2e6 --adapt-iters 100 --init-radius 0.1 --steps 40 --nuts-criterion stan2.23 > $O/fulldata_2e6.json 2> $O/fulldata_2e6.err || exit 6
python3 -c "import json; d=json.loads(open('$O/fulldata_2e6.json').read().strip().splitlines()[-1]); print('fulldata 2e6', d['value'], d['roofline']['achieved'], d.get('ess_per_sec'))"
timeout -k 10 400 python3 tools/bench_fulldata.py --rows-per-gpu 2.5e7 --steps 10 --warmup 2 > $O/fulldata_2.5e7.json 2> $O/fulldata_2.5e7.err || exit 7
python3 -c "import json; d=json.loads(open('$O/fulldata_2.5e7.json').read().strip().splitlines()[-1]); print('fulldata 2.5e7', d['value'], d['roofline']['achieved'], d['ms_per_step'])"
