#!/bin/bash
# round 5, call ah: final validation -- the full GPU suite (with the 64-chain cases at the C-ABI's
# largest d) and smoke; HBM bytes per launch of the GEMM passes (FETCH_SIZE, WRITE_SIZE in separate
# passes over the gemm_ab harness at configs[4]'s shape); the default bench line under a kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 500 --timeout-method thread tests > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit 7
python3 tools/pmc_gemm_traffic.py $O/pmc_fetch/pmc_counter_collection.csv $O/pmc_write/pmc_counter_collection.csv --rows-per-shard 2000000 --shards 8 --d 1000 --json $O/gemm_traffic.json
rm -rf $O/pmc_fetch $O/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 8
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweep16 --bench-json $O/bench.json --json $O/window.json
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -6 $O/stats.csv
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; c4=d['other_configs']['configs4_fulldata']; print('bench', d['value'], d['ess_per_sec'], r['frac'], r['avg_launch_ms'], r['traffic'], (d.get('configs1_schools') or {}).get('value'), 'c4', c4.get('value'), c4.get('ms_per_step'), (c4.get('roofline') or {}).get('frac'))"
rm -rf $O/prof
