#!/bin/bash
# round 5, call aq: validation after pass F's split stage schedule (on the round-5 pass F 128-row tiles, pass B
# 256-column blocks) -- the full GPU suite and smoke; SQ counters per pass F / pass B arm (gemm_ab
# harness, configs[4]'s shape); the default bench line (with its configs[4] sub-record) under a
# kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aq
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 500 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc_gemm -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_gemm.log 2>&1
rc=$?; echo "pmc gemm rc=$rc"; [ $rc -eq 0 ] || exit 6
python3 tools/pmc_arms.py $O/pmc_gemm/pmc_counter_collection.csv --json $O/gemm_pmc.json | tail -12
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 8
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweep16 --bench-json $O/bench.json --json $O/window.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -8 $O/stats.csv
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; c4=d['other_configs']['configs4_fulldata']; print('bench', d['value'], r['frac'], r['avg_launch_ms'], (d.get('configs1_schools') or {}).get('value'), 'c4', c4.get('value'), c4.get('ms_per_step'), (c4.get('roofline') or {}).get('frac'))"
rm -rf $O/prof
