cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench full rc=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o kt --output-format csv -- python3 tools/sweep_run.py --steps 40 > gpurun_out/prof_full.log 2>&1
rc=$?; echo "prof full rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/sweep_run.py --steps 6 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 tools/sweep_run.py --steps 6 > gpurun_out/pmc_write.log 2>&1
echo "pmc write rc=$?"
ls -R gpurun_out/pmc_fetch | head
