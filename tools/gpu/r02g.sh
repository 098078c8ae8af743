#!/bin/bash
# round 2, call g: Stan >= 2.23 U-turn checks -- parity/moment tests, combine inverse v5,
# headline bench with --nuts-criterion stan2.23
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_nuts.py tests/test_gpu_kernels.py -m gpu -q --timeout 250 --timeout-method thread -k "extended or schools or combine or transition or adaptive" > $O/r02g_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 3
timeout -k 10 120 python3 tools/combine_bench.py > $O/r02g_combine.json 2>&1 || exit 6
timeout -k 10 560 python3 bench.py --steps 20 --warmup 5 --nuts-criterion stan2.23 > $O/r02g_bench_223.json 2> $O/r02g_bench_223.err
echo "bench rc=$?"
timeout -k 10 400 python3 bench.py --family linear --rows 1e7 --d 50 --adapt-iters 1000 --steps 200 --warmup 5 --ess-draws 200 --no-cpu-baseline > $O/r02g_bench_linear.json 2> $O/r02g_bench_linear.err
echo "linear rc=$?"
