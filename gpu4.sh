cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -X faulthandler -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --rows 8e6 --steps 20 --warmup 2 --adapt-iters 60 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench small rc=$rc"; tail -1 gpurun_out/bench_small.log | cut -c1-900
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o kt --output-format csv -- python3 bench.py --rows 8e6 --steps 10 --warmup 1 --adapt-iters 20 --no-cpu-baseline > gpurun_out/prof_small.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof_small -name "*stats*" | head
