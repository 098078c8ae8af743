#!/bin/bash
# Default bench line with roofline.traffic for the launched sweep (k_sweepe at d = 100): the
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs), the bench, and the rocprofv3
# kernel-trace summary of the same bench command.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pmc_fetch -name "*counter_collection.csv" | head -1)
w=$(find gpurun_out/pmc_write -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$f" --write-csv "$w" --kernel k_sweepe --rows-per-shard 12500000 --d 100 --shards-per-gpu 8 --out gpurun_out/sweep_pmc.json
rc=$?; echo "pmc_traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/sweep_pmc.json profiles/sweep_pmc.json
timeout -k 10 700 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-3000
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof bench rc=$rc"; grep '"metric"' gpurun_out/prof_bench.log | cut -c1-400
find gpurun_out/prof_bench -name "*stats*"
exit $rc
