cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full2.log 2>&1
rc=$?; echo "bench full rc=$rc"; tail -1 gpurun_out/bench_full2.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof bench rc=$rc"; grep '"metric"' gpurun_out/prof_bench.log | cut -c1-300
