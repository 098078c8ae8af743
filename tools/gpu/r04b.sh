#!/bin/bash
# round 4, call b: validation of k_sweep16 in the product -- the full GPU suite and smoke; the
# default bench line under a kernel trace (timed window vs trace); PMC of the sweep (traffic, MFMA
# busy, VALU instructions, clock); the 8-GPU per-rank shape (1 shard of 1.25e7 rows) under a
# kernel trace; configs[2] under the reference's sampler configuration (Stan 2.19, jitter 0,
# iter = 2000).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 480 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 8
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweep16 --bench-json $O/bench.json --json $O/window.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -6 $O/stats.csv
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['bound'], r['frac'], r['avg_launch_ms'], d['cpu_baseline'] and d['cpu_baseline'].get('value'), d['combine']['gpu_ms'], (d.get('configs1_schools') or {}).get('value'))"
rm -rf $O/prof
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/pmc_fetch.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/pmc_write.log 2>&1 || exit 7
python3 tools/pmc_traffic.py $O/pmc_fetch/pmc_counter_collection.csv --write-csv $O/pmc_write/pmc_counter_collection.csv --kernel k_sweep16 --rows-per-shard 12500000 --d 100 --shards-per-gpu 8 --out $O/sweep_pmc.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/sweep16_ab 12500000 8 1 3 100 3 > $O/pmc_sq.log 2>&1 || exit 9
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/sweep16_pmc.json > $O/pmc_sq_summary.txt 2>&1; tail -30 $O/pmc_sq_summary.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --rows 1.25e7 --shards 1 --steps 400 --warmup 20 --no-cpu-baseline --second-criterion none --no-schools --no-accuracy > $O/bench_1shard.json 2> $O/bench_1shard.err
rc=$?; echo "1-shard rc=$rc"; [ $rc -eq 0 ] || exit 10
python3 tools/rocpd_summary.py window $O/prof1/run_results.db --kernel k_sweep16 --bench-json $O/bench_1shard.json --json $O/window_1shard.json
python3 tools/rocpd_summary.py stats $O/prof1/run_results.db > $O/stats_1shard.csv 2>&1; head -6 $O/stats_1shard.csv
rm -rf $O/prof1
timeout -k 10 240 python3 bench.py --family linear --rows 1e7 --d 50 --nuts-criterion stan2.19 --stepsize-jitter 0 --adapt-iters 1000 --ess-draws 1000 --second-criterion none --steps 20 --warmup 5 --no-schools > $O/bench_linear_refcfg.json 2> $O/bench_linear_refcfg.err
rc=$?; echo "linear refcfg rc=$rc"; tail -c 600 $O/bench_linear_refcfg.json
