cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"; tail -3 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --rows 8e6 --steps 20 --warmup 2 --adapt-iters 60 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench small rc=$rc"; tail -3 gpurun_out/bench_small.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1
echo "bench full rc=$?"; tail -4 gpurun_out/bench_full.log
