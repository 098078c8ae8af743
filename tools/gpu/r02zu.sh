#!/bin/bash
# round 2 re-entry: the headline workload with 64 chains per shard (two-pass GEMM sweep, d = 100)
# vs the default 16 (k_sweepe): gradient throughput and the clock the chip holds
set -o pipefail
mkdir -p gpurun_out/r02zu
O=gpurun_out/r02zu
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 bench.py --chains 64 --adapt-iters 60 --steps 60 --warmup 5 --ess-draws 20 --no-cpu-baseline --no-accuracy > $O/bench_c64.json 2> $O/bench_c64.err || exit 2
python3 -c "import json; d=json.loads(open('$O/bench_c64.json').read().strip().splitlines()[-1]); print('C64', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['setup_s'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/sweep_run.py --chains 64 --steps 12 > $O/sweep_run_c64.log 2>&1 || exit 3
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -5 $O/stats.csv
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 64 --steps 8 > $O/pmc.log 2>&1 || exit 4
echo pmc ok
