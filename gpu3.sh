cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -X faulthandler -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "leaves|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --rows 8e6 --steps 20 --warmup 2 --adapt-iters 60 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench small rc=$rc"; tail -3 gpurun_out/bench_small.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2>&1
echo "bench full rc=$?"; tail -6 gpurun_out/bench_full.log
