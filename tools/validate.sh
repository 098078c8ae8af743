#!/bin/bash
# The validation recipe of a tree, on one MI355X (run through gpurun from the repo root):
#   1. the GPU test suite and smoke();
#   2. k_sweep16's HBM traffic at the bench geometry: FETCH_SIZE and WRITE_SIZE in separate
#      --pmc passes over a fixed 6-step run (tools/sweep_run.py), corrected by tools/pmc_traffic.py
#      (FETCH_SIZE x 2 on gfx950, MI355X_MICROARCH.md) -> profiles/sweep_pmc.json, which the bench
#      line's roofline.traffic reads;
#   3. SQ / GRBM counters of the same run (MFMA busy, clock, waits; tools/pmc_arms.py);
#   4. the default bench line under a kernel trace: rocprofv3 --stats, and the k_sweep16
#      dispatches inside the line's timed window against the line's own event time
#      (tools/rocpd_summary.py window).
# Every GPU step has its own time limit; the first failure ends the script.
# usage: bash tools/validate.sh OUTDIR [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
O=$1
shift
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit 4
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$O/smoke.log"; [ $rc -eq 0 ] || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > "$O/pmc_fetch.log" 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > "$O/pmc_write.log" 2>&1 || exit 7
python3 tools/pmc_traffic.py "$O/pmc_fetch/pmc_counter_collection.csv" --write-csv "$O/pmc_write/pmc_counter_collection.csv" --kernel k_sweep16 --rows-per-shard 12500000 --d 100 --shards-per-gpu 8 --out "$O/sweep_pmc.json" || exit 8
cp "$O/sweep_pmc.json" profiles/sweep_pmc.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$O/pmc_sq" -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > "$O/pmc_sq.log" 2>&1 || exit 9
python3 tools/pmc_arms.py "$O/pmc_sq/pmc_counter_collection.csv" --json "$O/sweep16_pmc.json" > "$O/pmc_sq_summary.txt" 2>&1
rm -rf "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_sq"
timeout -k 10 800 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 10
python3 tools/rocpd_summary.py window "$O/prof/run_results.db" --kernel k_sweep16 --bench-json "$O/bench.json" --json "$O/window.json"
python3 tools/rocpd_summary.py stats "$O/prof/run_results.db" > "$O/kernel_stats.csv" 2>&1; head -8 "$O/kernel_stats.csv"
find "$O/prof" -name "*stats*.csv" -exec cp {} "$O/" \; 2>/dev/null
rm -rf "$O/prof"
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['frac'], r['avg_launch_ms'], r['traffic'])"
