#!/bin/bash
# round 5, call o: validation of the round-5 tree -- the full GPU suite and smoke; the sweep's HBM
# traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ counters per A/B arm; the default bench
# line under a kernel trace (timed window vs trace); the 8-schools stamped breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 500 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/pmc_fetch.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/pmc_write.log 2>&1 || exit 7
python3 tools/pmc_traffic.py $O/pmc_fetch/pmc_counter_collection.csv --write-csv $O/pmc_write/pmc_counter_collection.csv --kernel k_sweep16 --rows-per-shard 12500000 --d 100 --shards-per-gpu 8 --out $O/sweep_pmc.json
cp $O/sweep_pmc.json profiles/sweep_pmc.json
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/sweep16_ab 12500000 8 1 3 100 3 > $O/pmc_sq.log 2>&1 || exit 9
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/sweep16_pmc.json > $O/pmc_sq_summary.txt 2>&1; tail -8 $O/pmc_sq_summary.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 8
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweep16 --bench-json $O/bench.json --json $O/window.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -6 $O/stats.csv
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['bound'], r['frac'], r['avg_launch_ms'], r['traffic'], d['cpu_baseline'] and d['cpu_baseline'].get('value'), d['combine']['gpu_ms'], (d.get('configs1_schools') or {}).get('value'), (d.get('ess_second_criterion') or {}).get('ess_per_sec'))"
rm -rf $O/prof

timeout -k 10 200 python3 -u tools/schools_stamps.py run > $O/schools_stamps.json 2> $O/schools_stamps.err; echo "stamps rc=$?"
