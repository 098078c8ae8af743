#!/bin/bash
# round 3, call ad: k_sweepe as the product sweep for d = 50 -- kernel + NUTS tests, then the
# configs[2] bench line (linear N = 1e7, d = 50) under a kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 800 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --family linear --rows 1e7 --d 50 --steps 2000 --no-cpu-baseline > $O/bench_linear.json 2> $O/bench_linear.err || exit 2
python3 -c "import json; d=json.loads(open('$O/bench_linear.json').read().strip().splitlines()[-1]); print('linear', d['value'], d['ess_per_sec'], d['divergent'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['accuracy'].get('vs_fulldata_exact',{}).get('consensus'), (d.get('ess_second_criterion') or {}).get('ess_per_sec'))"
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -4 $O/stats.csv
rm -rf $O/prof
